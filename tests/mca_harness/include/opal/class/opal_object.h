/* TEST HARNESS ONLY: refcounted objects without class machinery. */
#ifndef HARNESS_OPAL_OBJECT_H
#define HARNESS_OPAL_OBJECT_H
#include <stdint.h>
#include <stdlib.h>
typedef struct opal_class_t opal_class_t;
typedef struct opal_object_t {
    opal_class_t *obj_class;
    volatile int32_t obj_reference_count;
} opal_object_t;
#define OBJ_CLASS_DECLARATION(t) extern int harness_class_##t
#define OBJ_NEW(type) ((type *) harness_obj_new(sizeof(type)))
#define OBJ_RETAIN(o) (((opal_object_t *) (o))->obj_reference_count++)
#define OBJ_RELEASE(o)                                                      \
    do {                                                                    \
        if (--((opal_object_t *) (o))->obj_reference_count == 0) free(o);   \
    } while (0)
static inline void *harness_obj_new(size_t n)
{
    opal_object_t *o = (opal_object_t *) calloc(1, n);
    o->obj_reference_count = 1;
    return o;
}
#endif
