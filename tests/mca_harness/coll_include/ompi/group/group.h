/* TEST HARNESS ONLY: the ompi_group_t fields and calls the glue uses
 * (ompi/group/group.h:80-95, 203-241).  A group lists its members as ranks
 * of the harness's world (grp_world NULL = the world itself, in order). */
#ifndef HARNESS_GROUP_H
#define HARNESS_GROUP_H
#include <stddef.h>
#ifndef MPI_UNDEFINED
#define MPI_UNDEFINED (-32766)
#endif
typedef struct ompi_group_t {
    int remote_peers;     /* stands in for ompi_group_have_remote_peers's proc scan */
    int grp_proc_count;
    const int *grp_world; /* member i is world rank grp_world[i] */
} ompi_group_t;
static inline int ompi_group_size(ompi_group_t *g) { return g->grp_proc_count; }
static inline int ompi_group_have_remote_peers(const ompi_group_t *g) { return g->remote_peers; }
static inline int ompi_group_translate_ranks(ompi_group_t *g1, int n, const int *r1,
                                             ompi_group_t *g2, int *r2)
{
    for (int i = 0; i < n; ++i) {
        const int w = g1->grp_world ? g1->grp_world[r1[i]] : r1[i];
        r2[i] = MPI_UNDEFINED;
        for (int j = 0; j < g2->grp_proc_count; ++j)
            if ((g2->grp_world ? g2->grp_world[j] : j) == w) r2[i] = j;
    }
    return 0;
}
#endif
