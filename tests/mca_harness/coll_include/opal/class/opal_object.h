/* TEST HARNESS ONLY: refcounted objects with constructor/destructor
 * (the subset of opal_object.h the coll glue uses). */
#ifndef HARNESS_OPAL_OBJECT_H
#define HARNESS_OPAL_OBJECT_H
#include <stdint.h>
#include <stdlib.h>
typedef struct opal_class_t {
    void (*ctor)(void *);
    void (*dtor)(void *);
} opal_class_t;
typedef struct opal_object_t {
    opal_class_t *obj_class;
    volatile int32_t obj_reference_count;
} opal_object_t;
#define OBJ_CLASS_DECLARATION(t) extern opal_class_t harness_class_##t
#define OBJ_CLASS_INSTANCE(t, parent, c, d) \
    opal_class_t harness_class_##t = {(void (*)(void *))(c), (void (*)(void *))(d)}
#define OBJ_NEW(type) ((type *) harness_obj_new(sizeof(type), &harness_class_##type))
#define OBJ_RETAIN(o) (((opal_object_t *) (o))->obj_reference_count++)
#define OBJ_RELEASE(o)                                                       \
    do {                                                                     \
        opal_object_t *o_ = (opal_object_t *) (o);                           \
        if (--o_->obj_reference_count == 0) {                                \
            if (o_->obj_class && o_->obj_class->dtor) o_->obj_class->dtor(o_); \
            free(o_);                                                        \
        }                                                                    \
    } while (0)
static inline void *harness_obj_new(size_t n, opal_class_t *cls)
{
    opal_object_t *o = (opal_object_t *) calloc(1, n);
    o->obj_class = cls;
    o->obj_reference_count = 1;
    if (cls && cls->ctor) cls->ctor(o);
    return o;
}
#endif
