/* TEST HARNESS ONLY: device buffers for op_select_harness.c. */
#define __HIP_PLATFORM_AMD__ 1
#include <hip/hip_runtime_api.h>

int harness_dev_alloc_copy(void **d, const void *h, size_t bytes)
{
    if (hipMalloc(d, bytes) != hipSuccess) return -1;
    return hipMemcpy(*d, h, bytes, hipMemcpyHostToDevice) == hipSuccess ? 0 : -1;
}

int harness_dev_copy_in(void *d, const void *h, size_t bytes)
{
    return hipMemcpy(d, h, bytes, hipMemcpyHostToDevice) == hipSuccess ? 0 : -1;
}

int harness_dev_copy_back(void *h, const void *d, size_t bytes)
{
    return hipMemcpy(h, d, bytes, hipMemcpyDeviceToHost) == hipSuccess ? 0 : -1;
}

int harness_dev_free(void *d)
{
    return hipFree(d) == hipSuccess ? 0 : -1;
}
