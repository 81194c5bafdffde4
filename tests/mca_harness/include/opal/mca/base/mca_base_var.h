/* TEST HARNESS ONLY */
#ifndef HARNESS_MCA_BASE_VAR_H
#define HARNESS_MCA_BASE_VAR_H
#include <stdbool.h>
#include <stdio.h>
#include <stdlib.h>
#include <string.h>
#include "ompi/mca/mca.h"
enum { MCA_BASE_VAR_TYPE_INT = 0 };
enum { OPAL_INFO_LVL_6 = 6, OPAL_INFO_LVL_9 = 9 };
enum { MCA_BASE_VAR_SCOPE_READONLY = 1 };
#ifndef OPAL_SUCCESS
#define OPAL_SUCCESS 0
#endif
typedef int mca_base_var_source_t;
static inline int mca_base_component_var_register(const mca_base_component_t *c, const char *name,
                                                  const char *help, int type, void *enumerator,
                                                  int bind, int flags, int level, int scope,
                                                  void *storage)
{
    (void) c; (void) name; (void) help; (void) type; (void) enumerator;
    (void) bind; (void) flags; (void) level; (void) scope; (void) storage;
    return 0;
}
/* Other components' variables, as the MCA variable system would hold them
 * after reading the environment (OMPI_MCA_<project-less full name>), which
 * is one of its sources: a variable is "registered" when its environment
 * variable is set.  Indices name a small table of storage cells: ints and
 * bools in harness_var_int, strings in harness_var_str. */
#define HARNESS_VARS 16
static char harness_var_name[HARNESS_VARS][96];
static int harness_var_int[HARNESS_VARS];
static bool harness_var_bool[HARNESS_VARS];
static char *harness_var_str[HARNESS_VARS];
static inline int mca_base_var_find(const char *project, const char *type, const char *comp,
                                    const char *name)
{
    char full[96];
    const char *v;
    int i;
    (void) project;
    snprintf(full, sizeof(full), "OMPI_MCA_%s_%s_%s", type, comp, name);
    v = getenv(full);
    if (NULL == v) return -1;
    for (i = 0; i < HARNESS_VARS && harness_var_name[i][0]; ++i)
        if (0 == strcmp(harness_var_name[i], full)) break;
    if (i == HARNESS_VARS) return -1;
    snprintf(harness_var_name[i], sizeof(harness_var_name[i]), "%s", full);
    harness_var_int[i] = atoi(v);
    harness_var_bool[i] = atoi(v) != 0 || 0 == strcmp(v, "true");
    harness_var_str[i] = (char *) v;
    return i;
}
/* the harness knows each variable's type by name: "use_*" are bools,
 * "*_filename" strings, the rest ints */
static inline int mca_base_var_get_value(int idx, const void *value, mca_base_var_source_t *source,
                                         const char **source_file)
{
    const char *n;
    (void) source; (void) source_file;
    if (idx < 0 || idx >= HARNESS_VARS || !harness_var_name[idx][0]) return -1;
    n = harness_var_name[idx];
    if (strstr(n, "_use_")) *(const void **) value = &harness_var_bool[idx];
    else if (strstr(n, "_filename")) *(const void **) value = &harness_var_str[idx];
    else *(const void **) value = &harness_var_int[idx];
    return 0;
}
#endif
