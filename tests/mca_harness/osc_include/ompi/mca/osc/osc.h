/* TEST HARNESS ONLY: the osc framework types with the reference's function
 * signatures and module slot order (ompi/mca/osc/osc.h:77-420). */
#ifndef HARNESS_OSC_H
#define HARNESS_OSC_H
#include <stdbool.h>
#include <stddef.h>
#include "ompi/mca/mca.h"
#include "ompi/request/request.h"
struct ompi_win_t;
struct ompi_communicator_t;
struct ompi_datatype_t;
struct ompi_op_t;
struct ompi_group_t;
struct opal_info_t;
#define W struct ompi_win_t *
#define DT struct ompi_datatype_t *
typedef int (*ompi_osc_base_component_init_fn_t)(bool, bool);
typedef int (*ompi_osc_base_component_finalize_fn_t)(void);
typedef int (*ompi_osc_base_component_query_fn_t)(W, void **, size_t, int,
                                                  struct ompi_communicator_t *,
                                                  struct opal_info_t *, int);
typedef int (*ompi_osc_base_component_select_fn_t)(W, void **, size_t, int,
                                                   struct ompi_communicator_t *,
                                                   struct opal_info_t *, int, int *);
typedef struct ompi_osc_base_component_2_0_0_t {
    mca_base_component_t osc_version;
    mca_base_component_data_t osc_data;
    ompi_osc_base_component_init_fn_t osc_init;
    ompi_osc_base_component_query_fn_t osc_query;
    ompi_osc_base_component_select_fn_t osc_select;
    ompi_osc_base_component_finalize_fn_t osc_finalize;
} ompi_osc_base_component_2_0_0_t;
typedef ompi_osc_base_component_2_0_0_t ompi_osc_base_component_t;
typedef int (*ompi_osc_base_module_win_shared_query_fn_t)(W, int, size_t *, int *, void *);
typedef int (*ompi_osc_base_module_win_attach_fn_t)(W, void *, size_t);
typedef int (*ompi_osc_base_module_win_detach_fn_t)(W, const void *);
typedef int (*ompi_osc_base_module_free_fn_t)(W);
typedef int (*ompi_osc_base_module_put_fn_t)(const void *, int, DT, int, ptrdiff_t, int, DT, W);
typedef int (*ompi_osc_base_module_get_fn_t)(void *, int, DT, int, ptrdiff_t, int, DT, W);
typedef int (*ompi_osc_base_module_accumulate_fn_t)(const void *, int, DT, int, ptrdiff_t, int, DT,
                                                   struct ompi_op_t *, W);
typedef int (*ompi_osc_base_module_compare_and_swap_fn_t)(const void *, const void *, void *, DT,
                                                          int, ptrdiff_t, W);
typedef int (*ompi_osc_base_module_fetch_and_op_fn_t)(const void *, void *, DT, int, ptrdiff_t,
                                                      struct ompi_op_t *, W);
typedef int (*ompi_osc_base_module_get_accumulate_fn_t)(const void *, int, DT, void *, int, DT,
                                                        int, ptrdiff_t, int, DT,
                                                        struct ompi_op_t *, W);
typedef int (*ompi_osc_base_module_rput_fn_t)(const void *, int, DT, int, ptrdiff_t, int, DT, W,
                                             ompi_request_t **);
typedef int (*ompi_osc_base_module_rget_fn_t)(void *, int, DT, int, ptrdiff_t, int, DT, W,
                                             ompi_request_t **);
typedef int (*ompi_osc_base_module_raccumulate_fn_t)(const void *, int, DT, int, ptrdiff_t, int,
                                                    DT, struct ompi_op_t *, W, ompi_request_t **);
typedef int (*ompi_osc_base_module_rget_accumulate_fn_t)(const void *, int, DT, void *, int, DT,
                                                        int, ptrdiff_t, int, DT,
                                                        struct ompi_op_t *, W, ompi_request_t **);
typedef int (*ompi_osc_base_module_fence_fn_t)(int, W);
typedef int (*ompi_osc_base_module_start_fn_t)(struct ompi_group_t *, int, W);
typedef int (*ompi_osc_base_module_complete_fn_t)(W);
typedef int (*ompi_osc_base_module_post_fn_t)(struct ompi_group_t *, int, W);
typedef int (*ompi_osc_base_module_wait_fn_t)(W);
typedef int (*ompi_osc_base_module_test_fn_t)(W, int *);
typedef int (*ompi_osc_base_module_lock_fn_t)(int, int, int, W);
typedef int (*ompi_osc_base_module_unlock_fn_t)(int, W);
typedef int (*ompi_osc_base_module_lock_all_fn_t)(int, W);
typedef int (*ompi_osc_base_module_unlock_all_fn_t)(W);
typedef int (*ompi_osc_base_module_sync_fn_t)(W);
typedef int (*ompi_osc_base_module_flush_fn_t)(int, W);
typedef int (*ompi_osc_base_module_flush_all_fn_t)(W);
typedef int (*ompi_osc_base_module_flush_local_fn_t)(int, W);
typedef int (*ompi_osc_base_module_flush_local_all_fn_t)(W);
#undef W
#undef DT
typedef struct ompi_osc_base_module_3_0_0_t {
    ompi_osc_base_module_win_shared_query_fn_t osc_win_shared_query;
    ompi_osc_base_module_win_attach_fn_t osc_win_attach;
    ompi_osc_base_module_win_detach_fn_t osc_win_detach;
    ompi_osc_base_module_free_fn_t osc_free;
    ompi_osc_base_module_put_fn_t osc_put;
    ompi_osc_base_module_get_fn_t osc_get;
    ompi_osc_base_module_accumulate_fn_t osc_accumulate;
    ompi_osc_base_module_compare_and_swap_fn_t osc_compare_and_swap;
    ompi_osc_base_module_fetch_and_op_fn_t osc_fetch_and_op;
    ompi_osc_base_module_get_accumulate_fn_t osc_get_accumulate;
    ompi_osc_base_module_rput_fn_t osc_rput;
    ompi_osc_base_module_rget_fn_t osc_rget;
    ompi_osc_base_module_raccumulate_fn_t osc_raccumulate;
    ompi_osc_base_module_rget_accumulate_fn_t osc_rget_accumulate;
    ompi_osc_base_module_fence_fn_t osc_fence;
    ompi_osc_base_module_start_fn_t osc_start;
    ompi_osc_base_module_complete_fn_t osc_complete;
    ompi_osc_base_module_post_fn_t osc_post;
    ompi_osc_base_module_wait_fn_t osc_wait;
    ompi_osc_base_module_test_fn_t osc_test;
    ompi_osc_base_module_lock_fn_t osc_lock;
    ompi_osc_base_module_unlock_fn_t osc_unlock;
    ompi_osc_base_module_lock_all_fn_t osc_lock_all;
    ompi_osc_base_module_unlock_all_fn_t osc_unlock_all;
    ompi_osc_base_module_sync_fn_t osc_sync;
    ompi_osc_base_module_flush_fn_t osc_flush;
    ompi_osc_base_module_flush_all_fn_t osc_flush_all;
    ompi_osc_base_module_flush_local_fn_t osc_flush_local;
    ompi_osc_base_module_flush_local_all_fn_t osc_flush_local_all;
} ompi_osc_base_module_3_0_0_t;
typedef ompi_osc_base_module_3_0_0_t ompi_osc_base_module_t;
#define OMPI_OSC_BASE_VERSION_3_0_0 OMPI_MCA_BASE_VERSION_2_1_0("osc", 3, 0, 0)
#endif
