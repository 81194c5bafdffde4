/* TEST HARNESS ONLY: opal_info_t as a key/value list, opal_info_get_bool
 * (opal/util/info.h). */
#ifndef HARNESS_OPAL_INFO_H
#define HARNESS_OPAL_INFO_H
#include <stdbool.h>
#include <stddef.h>
#include <string.h>
typedef struct opal_info_t {
    const char *key;
    const char *value;
    const struct opal_info_t *next;  /* further entries (NULL: none) */
} opal_info_t;
static inline int opal_info_get_bool(opal_info_t *info, const char *key, bool *value, int *flag)
{
    const opal_info_t *e = info;
    while (e && !(e->key && 0 == strcmp(e->key, key))) e = e->next;
    *flag = NULL != e;
    if (*flag) *value = 0 == strcmp(e->value, "true") || 0 == strcmp(e->value, "1");
    return 0;
}
#endif
