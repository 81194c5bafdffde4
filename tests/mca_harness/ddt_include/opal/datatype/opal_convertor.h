/* TEST HARNESS ONLY: opal_convertor_t and its entry points
 * (opal/datatype/opal_convertor.h:40-147), restated with the reference's
 * full field list and order (:88-124), including the fields that exist only
 * when the build has OPAL_CUDA_SUPPORT; the harness is compiled both ways
 * (build_ddt.sh) so the seam is exercised on a ROCm-only layout too.  The
 * harness supplies a minimal prepare / pack / unpack / set_position
 * (ddt_harness.c). */
#ifndef HARNESS_OPAL_CONVERTOR_H
#define HARNESS_OPAL_CONVERTOR_H
#include <stddef.h>
#include <stdint.h>
#include <sys/uio.h>

#include "opal/datatype/opal_datatype.h"

#ifndef OPAL_CUDA_SUPPORT
#define OPAL_CUDA_SUPPORT 0
#endif

#define CONVERTOR_DATATYPE_MASK 0x0000FFFF
#define CONVERTOR_SEND_CONVERSION 0x00010000
#define CONVERTOR_RECV 0x00020000
#define CONVERTOR_SEND 0x00040000
#define CONVERTOR_HOMOGENEOUS 0x00080000
#define CONVERTOR_NO_OP 0x00100000
#define CONVERTOR_WITH_CHECKSUM 0x00200000
#define CONVERTOR_CUDA 0x00400000
#define CONVERTOR_CUDA_ASYNC 0x00800000
#define CONVERTOR_TYPE_MASK 0x10FF0000
#define CONVERTOR_STATE_START 0x01000000
#define CONVERTOR_STATE_COMPLETE 0x02000000
#define CONVERTOR_STATE_ALLOC 0x04000000
#define CONVERTOR_COMPLETED 0x08000000
#define CONVERTOR_CUDA_UNIFIED 0x10000000
#define CONVERTOR_HAS_REMOTE_SIZE 0x20000000
#define CONVERTOR_SKIP_CUDA_INIT 0x40000000

typedef struct opal_convertor_t opal_convertor_t;
typedef int32_t (*convertor_advance_fct_t)(opal_convertor_t *pConvertor, struct iovec *iov,
                                           uint32_t *out_size, size_t *max_data);
typedef void *(*memalloc_fct_t)(size_t *pLength, void *userdata);
typedef void *(*memcpy_fct_t)(void *dest, const void *src, size_t n, opal_convertor_t *pConvertor);

struct opal_convertor_master_t;

struct dt_stack_t {
    int32_t index;
    int16_t type;
    int16_t padding;
    size_t count;
    ptrdiff_t disp;
};
typedef struct dt_stack_t dt_stack_t;

#define DT_STATIC_STACK_SIZE 5

struct opal_convertor_t {
    opal_object_t super;
    uint32_t remoteArch;
    uint32_t flags;
    size_t local_size;
    size_t remote_size;
    const opal_datatype_t *pDesc;
    const dt_type_desc_t *use_desc;
    opal_datatype_count_t count;
    uint32_t stack_size;
    unsigned char *pBaseBuf;
    dt_stack_t *pStack;
    convertor_advance_fct_t fAdvance;
    struct opal_convertor_master_t *master;
    uint32_t stack_pos;
    size_t partial_length;
    size_t bConverted;
    uint32_t checksum;
    uint32_t csum_ui1;
    size_t csum_ui2;
    dt_stack_t static_stack[DT_STATIC_STACK_SIZE];
#if OPAL_CUDA_SUPPORT
    memcpy_fct_t cbmemcpy;
    void *stream;
#endif
};

int32_t opal_convertor_pack(opal_convertor_t *pConv, struct iovec *iov, uint32_t *out_size,
                            size_t *max_data);
int32_t opal_convertor_unpack(opal_convertor_t *pConv, struct iovec *iov, uint32_t *out_size,
                              size_t *max_data);
int32_t opal_convertor_prepare_for_send(opal_convertor_t *convertor,
                                        const struct opal_datatype_t *datatype, size_t count,
                                        const void *pUserBuf);
int32_t opal_convertor_prepare_for_recv(opal_convertor_t *convertor,
                                        const struct opal_datatype_t *datatype, size_t count,
                                        const void *pUserBuf);
int32_t opal_convertor_set_position(opal_convertor_t *convertor, size_t *position);
#endif
