/* TEST HARNESS ONLY: opal_info_t as a key/value list, opal_info_get_bool
 * (opal/util/info.h). */
#ifndef HARNESS_OPAL_INFO_H
#define HARNESS_OPAL_INFO_H
#include <stdbool.h>
#include <string.h>
typedef struct opal_info_t {
    const char *key;   /* one entry is enough for the harness */
    const char *value;
} opal_info_t;
static inline int opal_info_get_bool(opal_info_t *info, const char *key, bool *value, int *flag)
{
    *flag = info && info->key && 0 == strcmp(info->key, key);
    if (*flag) *value = 0 == strcmp(info->value, "true") || 0 == strcmp(info->value, "1");
    return 0;
}
#endif
