/* TEST HARNESS ONLY: opal_convertor_t and its entry points
 * (opal/datatype/opal_convertor.h:40-147), restated; the harness supplies a
 * minimal prepare / pack / unpack (ddt_harness.c). */
#ifndef HARNESS_OPAL_CONVERTOR_H
#define HARNESS_OPAL_CONVERTOR_H
#include <stddef.h>
#include <stdint.h>
#include <sys/uio.h>

#include "opal/datatype/opal_datatype.h"

#define CONVERTOR_SEND_CONVERSION 0x00010000
#define CONVERTOR_RECV 0x00020000
#define CONVERTOR_SEND 0x00040000
#define CONVERTOR_HOMOGENEOUS 0x00080000
#define CONVERTOR_NO_OP 0x00100000
#define CONVERTOR_WITH_CHECKSUM 0x00200000
#define CONVERTOR_CUDA 0x00400000
#define CONVERTOR_CUDA_ASYNC 0x00800000
#define CONVERTOR_COMPLETED 0x08000000

typedef struct opal_convertor_t opal_convertor_t;
typedef int32_t (*convertor_advance_fct_t)(opal_convertor_t *pConvertor, struct iovec *iov,
                                           uint32_t *out_size, size_t *max_data);
typedef void *(*memcpy_fct_t)(void *dest, const void *src, size_t n, opal_convertor_t *pConvertor);

struct opal_convertor_t {
    opal_object_t super;
    uint32_t remoteArch;
    uint32_t flags;
    size_t local_size;
    size_t remote_size;
    const opal_datatype_t *pDesc;
    const dt_type_desc_t *use_desc;
    size_t count;
    unsigned char *pBaseBuf;
    convertor_advance_fct_t fAdvance;
    size_t bConverted;
    memcpy_fct_t cbmemcpy;
    void *stream;
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
#endif
