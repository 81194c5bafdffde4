/* TEST HARNESS ONLY: the ompi_win_t field the osc glue sets (ompi/win/win.h:109). */
#ifndef HARNESS_OMPI_WIN_H
#define HARNESS_OMPI_WIN_H
struct ompi_osc_base_module_3_0_0_t;
typedef struct ompi_win_t {
    struct ompi_osc_base_module_3_0_0_t *w_osc_module;
} ompi_win_t;
#endif
