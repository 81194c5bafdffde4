/* TEST HARNESS ONLY */
#ifndef HARNESS_MCA_BASE_VAR_H
#define HARNESS_MCA_BASE_VAR_H
#include "ompi/mca/mca.h"
enum { MCA_BASE_VAR_TYPE_INT = 0 };
enum { OPAL_INFO_LVL_6 = 6, OPAL_INFO_LVL_9 = 9 };
enum { MCA_BASE_VAR_SCOPE_READONLY = 1 };
static inline int mca_base_component_var_register(const mca_base_component_t *c, const char *name,
                                                  const char *help, int type, void *enumerator,
                                                  int bind, int flags, int level, int scope,
                                                  void *storage)
{
    (void) c; (void) name; (void) help; (void) type; (void) enumerator;
    (void) bind; (void) flags; (void) level; (void) scope; (void) storage;
    return 0;
}
#endif
