/* TEST HARNESS ONLY: the convertor's GPU function table
 * (opal/datatype/opal_datatype_cuda.h:16-31), restated. */
#ifndef HARNESS_OPAL_DATATYPE_CUDA_H
#define HARNESS_OPAL_DATATYPE_CUDA_H
#include <stddef.h>

#include "opal/datatype/opal_convertor.h"

struct opal_common_cuda_function_table {
    int (*gpu_is_gpu_buffer)(const void *, opal_convertor_t *);
    int (*gpu_cu_memcpy_async)(void *, const void *, size_t, opal_convertor_t *);
    int (*gpu_cu_memcpy)(void *, const void *, size_t);
    int (*gpu_memmove)(void *, void *, size_t);
};
typedef struct opal_common_cuda_function_table opal_common_cuda_function_table_t;

void mca_cuda_convertor_init(opal_convertor_t *convertor, const void *pUserBuf);
void opal_cuda_add_initialization_function(int (*fptr)(opal_common_cuda_function_table_t *));
#endif
