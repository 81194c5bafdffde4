/*
 * Convertor offload for device buffers (see opal_datatype_rocm.h).
 *
 * The reference converts a device buffer by walking opt_desc on the host
 * and issuing one cuMemcpy per contiguous run (opal_generic_simple_pack,
 * opal_datatype_pack.c:235-370, with cbmemcpy = opal_cuda_memcpy,
 * opal_datatype_cuda.c:121-145).  Here opt_desc is flattened once per
 * datatype into a device program of {count, blocklen, stride, disp}
 * elements (include/ompi_amd_ddt.h) and each fAdvance call is one kernel
 * launch over all the iovec entries it is given.
 */
#include <pthread.h>
#include <stddef.h>
#include <stdint.h>
#include <stdlib.h>
#include <string.h>

#include "opal/datatype/opal_convertor.h"
#include "opal/datatype/opal_datatype.h"
#if OPAL_CUDA_SUPPORT
#include "opal/datatype/opal_datatype_cuda.h"
#endif
#include "opal/datatype/opal_datatype_internal.h"

#include "ompi_amd.h"
#include "ompi_amd_ddt.h"
#include "opal_datatype_rocm.h"

_Static_assert(sizeof(struct iovec) == sizeof(ompi_amd_iovec_t) &&
                   offsetof(struct iovec, iov_base) == offsetof(ompi_amd_iovec_t, iov_base) &&
                   offsetof(struct iovec, iov_len) == offsetof(ompi_amd_iovec_t, iov_len),
               "ompi_amd_iovec_t mirrors struct iovec");

/* The convertor's stream exists only in an OPAL_CUDA_SUPPORT build
 * (opal_convertor.h:120-123); otherwise the calling thread's library
 * stream (ompi_amd_set_thread_stream, NULL = the per-thread default). */
static void *conv_stream(const opal_convertor_t *c)
{
#if OPAL_CUDA_SUPPORT
    return c->stream;
#else
    (void) c;
    return NULL;
#endif
}

#if OPAL_CUDA_SUPPORT
/* ------------------------------------------------- GPU function table */

/* mca_common_cuda_is_gpu_buffer (common_cuda.c:1739-1792) */
static int rocm_is_gpu_buffer(const void *buf, opal_convertor_t *convertor)
{
    (void)convertor;
    return ompi_amd_is_device_pointer(buf);
}

/* mca_common_cuda_cu_memcpy_async (common_cuda.c:1862-1871): on the
 * convertor's stream */
static int rocm_memcpy_async(void *dst, const void *src, size_t n, opal_convertor_t *convertor)
{
    return ompi_amd_memcpy_async(dst, src, n, convertor ? conv_stream(convertor) : NULL) == 0 ? 0 : -1;
}

static int rocm_memcpy(void *dst, const void *src, size_t n)
{
    return ompi_amd_memcpy(dst, src, n) == 0 ? 0 : -1;
}

static int rocm_memmove(void *dst, void *src, size_t n)
{
    return ompi_amd_memmove(dst, src, n) == 0 ? 0 : -1;
}

int mca_common_rocm_fill_table(opal_common_cuda_function_table_t *ftable)
{
    if (!ftable || ompi_amd_device_count() <= 0) return -1;  /* OPAL_ERROR: no GPU support */
    ftable->gpu_is_gpu_buffer = &rocm_is_gpu_buffer;
    ftable->gpu_cu_memcpy_async = &rocm_memcpy_async;
    ftable->gpu_cu_memcpy = &rocm_memcpy;
    ftable->gpu_memmove = &rocm_memmove;
    return 0;
}
#endif /* OPAL_CUDA_SUPPORT */

/* ------------------------------------------ opt_desc -> device program */

typedef struct {
    ompi_amd_ddt_elem_t *e;
    int n, cap;
} elem_vec;

#define FLAT_MAX_ELEMS 4096 /* larger unrolled descriptions stay on the host path */

static int push(elem_vec *v, int64_t count, int64_t blen, int64_t stride, int64_t disp)
{
    if (count <= 0 || blen <= 0) return 0;
    if (count == 1) stride = blen;
    else if (stride == blen) { blen *= count; count = 1; stride = blen; }  /* one run */
    if (v->n > 0) {  /* a run that continues the previous one */
        ompi_amd_ddt_elem_t *p = &v->e[v->n - 1];
        if (p->count == 1 && count == 1 && p->disp + p->blocklen == disp) {
            p->blocklen += blen;
            p->stride = p->blocklen;
            return 0;
        }
    }
    if (v->n == FLAT_MAX_ELEMS) return -1;
    if (v->n == v->cap) {
        int cap = v->cap ? 2 * v->cap : 16;
        ompi_amd_ddt_elem_t *e = realloc(v->e, (size_t)cap * sizeof(*e));
        if (!e) return -1;
        v->e = e;
        v->cap = cap;
    }
    v->e[v->n++] = (ompi_amd_ddt_elem_t){count, blen, stride, disp};
    return 0;
}

/* Elements of desc[i0, i1) (typemap order) at byte offset `base`. */
static int flatten(const dt_elem_desc_t *d, uint32_t i0, uint32_t i1, ptrdiff_t base, elem_vec *out,
                   int depth)
{
    if (depth > 16) return -1;
    for (uint32_t i = i0; i < i1;) {
        const uint16_t type = d[i].elem.common.type;
        if (type == OPAL_DATATYPE_LOOP) {
            /* loop: items entries, the last one its END_LOOP; loops
             * repetitions extent bytes apart (opal_datatype_pack.c:303-351) */
            const uint32_t items = d[i].loop.items, loops = d[i].loop.loops;
            const ptrdiff_t ext = d[i].loop.extent;
            elem_vec body = {0};
            if (items < 1 || i + items > i1 ||
                flatten(d, i + 1, i + items, 0, &body, depth + 1) != 0) {
                free(body.e);
                return -1;
            }
            int rc = 0;
            if (body.n == 1 && body.e[0].count == 1) {
                rc = push(out, loops, body.e[0].blocklen, ext, base + body.e[0].disp);
            } else if (body.n == 1 && body.e[0].count * body.e[0].stride == ext) {
                rc = push(out, (int64_t)loops * body.e[0].count, body.e[0].blocklen, body.e[0].stride,
                          base + body.e[0].disp);
            } else if ((int64_t)loops * body.n <= FLAT_MAX_ELEMS) {
                for (uint32_t r = 0; r < loops && rc == 0; ++r)
                    for (int k = 0; k < body.n && rc == 0; ++k)
                        rc = push(out, body.e[k].count, body.e[k].blocklen, body.e[k].stride,
                                  base + (ptrdiff_t)r * ext + body.e[k].disp);
            } else {
                rc = -1;
            }
            free(body.e);
            if (rc != 0) return -1;
            i += items + 1;
        } else if (type == OPAL_DATATYPE_END_LOOP) {
            ++i;  /* the description's closing marker */
        } else if (d[i].elem.common.flags & OPAL_DATATYPE_FLAG_DATA) {
            /* count blocks of blocklen basic elements, extent bytes apart */
            if (type >= OPAL_DATATYPE_MAX_PREDEFINED || !opal_datatype_basicDatatypes[type]) return -1;
            const int64_t bsz = (int64_t)opal_datatype_basicDatatypes[type]->size;
            if (push(out, (int64_t)d[i].elem.count, (int64_t)d[i].elem.blocklen * bsz,
                     (int64_t)d[i].elem.extent, (int64_t)(base + d[i].elem.disp)) != 0)
                return -1;
            ++i;
        } else {
            ++i;  /* LB / UB markers carry no data */
        }
    }
    return 0;
}

/* ------------------------------------------------------- program cache */

typedef struct {
    const opal_datatype_t *dt;
    size_t size, used;
    ptrdiff_t lb, ub;
    dt_elem_desc_t *copy;  /* the description the program was built from */
    ompi_amd_ddt_t *prog;  /* NULL: not offloadable */
} prog_entry;

#define CACHE_MAX 256
static prog_entry g_cache[CACHE_MAX];
static int g_ncache, g_next_victim;
static ompi_amd_ddt_t **g_retired;  /* evicted programs a convertor may still use */
static int g_nretired, g_capretired;
static pthread_mutex_t g_lock = PTHREAD_MUTEX_INITIALIZER;

static int same_desc(const prog_entry *e, const opal_datatype_t *dt)
{
    return e->dt == dt && e->size == dt->size && e->lb == dt->lb && e->ub == dt->ub &&
           e->used == dt->opt_desc.used &&
           0 == memcmp(e->copy, dt->opt_desc.desc, e->used * sizeof(dt_elem_desc_t));
}

static void retire(ompi_amd_ddt_t *p)
{
    if (!p) return;
    if (g_nretired == g_capretired) {
        int cap = g_capretired ? 2 * g_capretired : 16;
        ompi_amd_ddt_t **r = realloc(g_retired, (size_t)cap * sizeof(*r));
        if (!r) return;  /* leak it: never destroy a program a convertor may use */
        g_retired = r;
        g_capretired = cap;
    }
    g_retired[g_nretired++] = p;
}

static ompi_amd_ddt_t *build(const opal_datatype_t *dt)
{
    elem_vec v = {0};
    ompi_amd_ddt_t *prog = NULL;
    if (flatten(dt->opt_desc.desc, 0, (uint32_t)dt->opt_desc.used, 0, &v, 0) == 0 && v.n > 0) {
        if (ompi_amd_ddt_create_elems(v.e, v.n, (int64_t)(dt->ub - dt->lb), &prog) != 0) prog = NULL;
        if (prog && ompi_amd_ddt_size(prog) != dt->size) {  /* the flattening must cover the type */
            ompi_amd_ddt_destroy(prog);
            prog = NULL;
        }
    }
    free(v.e);
    return prog;
}

/* The program of dt (built on first use); validated against a copy of the
 * description so that a datatype freed and re-created at the same address
 * never runs on the old program. */
static ompi_amd_ddt_t *program_of(const opal_datatype_t *dt, int validate)
{
    pthread_mutex_lock(&g_lock);
    for (int i = 0; i < g_ncache; ++i) {
        if (g_cache[i].dt != dt) continue;
        if (!validate || same_desc(&g_cache[i], dt)) {
            ompi_amd_ddt_t *p = g_cache[i].prog;
            pthread_mutex_unlock(&g_lock);
            return p;
        }
        retire(g_cache[i].prog);  /* stale: rebuild in place */
        free(g_cache[i].copy);
        g_cache[i] = g_cache[--g_ncache];
        break;
    }
    prog_entry e = {dt, dt->size, dt->opt_desc.used, dt->lb, dt->ub, NULL, NULL};
    e.copy = malloc(e.used * sizeof(dt_elem_desc_t) + 1);
    if (e.copy) {
        memcpy(e.copy, dt->opt_desc.desc, e.used * sizeof(dt_elem_desc_t));
        e.prog = build(dt);
        int slot = g_ncache;
        if (g_ncache == CACHE_MAX) {
            slot = g_next_victim;
            g_next_victim = (g_next_victim + 1) % CACHE_MAX;
            retire(g_cache[slot].prog);
            free(g_cache[slot].copy);
        } else {
            ++g_ncache;
        }
        g_cache[slot] = e;
    }
    pthread_mutex_unlock(&g_lock);
    return e.prog;
}

int opal_rocm_program_cache_size(void)
{
    pthread_mutex_lock(&g_lock);
    const int n = g_ncache;
    pthread_mutex_unlock(&g_lock);
    return n;
}

void opal_rocm_program_cache_clear(void)
{
    pthread_mutex_lock(&g_lock);
    for (int i = 0; i < g_ncache; ++i) {
        if (g_cache[i].prog) ompi_amd_ddt_destroy(g_cache[i].prog);
        free(g_cache[i].copy);
    }
    for (int i = 0; i < g_nretired; ++i) ompi_amd_ddt_destroy(g_retired[i]);
    free(g_retired);
    g_retired = NULL;
    g_nretired = g_capretired = g_ncache = g_next_victim = 0;
    pthread_mutex_unlock(&g_lock);
}

/* ------------------------------------------------------ advance step */

static int32_t advance(opal_convertor_t *conv, struct iovec *iov, uint32_t *out_size,
                       size_t *max_data, int unpack)
{
    ompi_amd_ddt_t *prog = program_of(conv->pDesc, 0);
    if (!prog) return -1;
    const int rc = unpack
        ? ompi_amd_ddt_unpack_iov(prog, conv->count, conv->pBaseBuf, conv->bConverted,
                                  (ompi_amd_iovec_t *)iov, out_size, max_data, conv_stream(conv))
        : ompi_amd_ddt_pack_iov(prog, conv->count, conv->pBaseBuf, conv->bConverted,
                                (ompi_amd_iovec_t *)iov, out_size, max_data, conv_stream(conv));
    if (rc < 0) return -1;
    /* synchronous unless the PML runs the convertor asynchronously and
     * waits on its stream itself (CONVERTOR_CUDA_ASYNC, set only by a CUDA
     * build's opal_cuda_set_copy_function_async) */
    if (!(conv->flags & CONVERTOR_CUDA_ASYNC) && ompi_amd_stream_synchronize(conv_stream(conv)) != 0)
        return -1;
    conv->bConverted += *max_data;
    if (rc == 1) conv->flags |= CONVERTOR_COMPLETED;
    return rc;
}

int32_t opal_rocm_pack(opal_convertor_t *convertor, struct iovec *iov, uint32_t *out_size,
                       size_t *max_data)
{
    return advance(convertor, iov, out_size, max_data, 0);
}

int32_t opal_rocm_unpack(opal_convertor_t *convertor, struct iovec *iov, uint32_t *out_size,
                         size_t *max_data)
{
    return advance(convertor, iov, out_size, max_data, 1);
}

#if !OPAL_CUDA_SUPPORT
/* A ROCm-only build has no cbmemcpy hook (opal_convertor.h:120-123): the
 * reference's host walker would memcpy the device buffer with the CPU.  A
 * device buffer whose datatype has no device program (more than
 * FLAT_MAX_ELEMS flattened elements, a leaf that is not predefined) gets
 * this fAdvance instead: the conversion fails with -1 (the contract's error
 * return) and nothing is read or written. */
int32_t opal_rocm_refuse(opal_convertor_t *convertor, struct iovec *iov, uint32_t *out_size,
                         size_t *max_data)
{
    (void) convertor;
    (void) iov;
    *out_size = 0;
    *max_data = 0;
    return -1;
}
#endif

/* The first byte the conversion touches is device memory (the reference's
 * mca_cuda_convertor_init asks the same of pUserBuf, opal_datatype_cuda.c:
 * 44-60; the true lower bound keeps a type with a negative lb inside the
 * allocation). */
#if !OPAL_CUDA_SUPPORT
static int device_buffer(const opal_convertor_t *c)
{
    if (NULL == c->pBaseBuf || NULL == c->pDesc) return 0;
    return ompi_amd_is_device_pointer(c->pBaseBuf + c->pDesc->true_lb);
}
#endif

int opal_rocm_convertor_select(opal_convertor_t *convertor)
{
    const uint32_t f = convertor->flags;
    if ((f & (CONVERTOR_NO_OP | CONVERTOR_COMPLETED | CONVERTOR_SKIP_CUDA_INIT)) ||
        !(f & CONVERTOR_HOMOGENEOUS) || (f & CONVERTOR_WITH_CHECKSUM))
        return 0;
#if OPAL_CUDA_SUPPORT
    /* a CUDA-support build flagged device buffers already (mca_cuda_convertor_init) */
    if (!(f & CONVERTOR_CUDA)) return 0;
#else
    /* a ROCm-only build: this seam asks the runtime itself */
    if (!device_buffer(convertor)) return 0;
    if (!program_of(convertor->pDesc, 1)) {  /* never the CPU on device memory */
        convertor->fAdvance = opal_rocm_refuse;
        return 1;
    }
#endif
    if (!program_of(convertor->pDesc, 1)) return 0;
    convertor->fAdvance = (f & CONVERTOR_SEND) ? opal_rocm_pack : opal_rocm_unpack;
    return 1;
}

int opal_rocm_convertor_owns(const opal_convertor_t *convertor)
{
#if !OPAL_CUDA_SUPPORT
    if (convertor->fAdvance == opal_rocm_refuse) return 1;
#endif
    return convertor->fAdvance == opal_rocm_pack || convertor->fAdvance == opal_rocm_unpack;
}

/* Packed offset, within desc[i0, i1) (r bytes into its packed stream), of
 * the start of the predefined element that holds byte r. */
static size_t snap_in(const dt_elem_desc_t *d, uint32_t i0, uint32_t i1, size_t r, int depth)
{
    size_t at = 0;
    for (uint32_t i = i0; i < i1 && depth < 16;) {
        const uint16_t type = d[i].elem.common.type;
        if (type == OPAL_DATATYPE_LOOP) {
            const uint32_t items = d[i].loop.items;
            if (items < 1 || i + items >= i1) return at;
            const size_t body = d[i + items].end_loop.size, total = body * d[i].loop.loops;
            if (body && r < at + total) {
                const size_t k = (r - at) / body;
                return at + k * body + snap_in(d, i + 1, i + items, (r - at) - k * body, depth + 1);
            }
            at += total;
            i += items + 1;
        } else if (type == OPAL_DATATYPE_END_LOOP) {
            ++i;
        } else if ((d[i].elem.common.flags & OPAL_DATATYPE_FLAG_DATA) &&
                   type < OPAL_DATATYPE_MAX_PREDEFINED && opal_datatype_basicDatatypes[type]) {
            const size_t bsz = opal_datatype_basicDatatypes[type]->size;
            const size_t bytes = (size_t)d[i].elem.count * d[i].elem.blocklen * bsz;
            if (bsz && r < at + bytes) return at + (r - at) / bsz * bsz;
            at += bytes;
            ++i;
        } else {
            ++i;
        }
    }
    return at;
}

/* opal_convertor_set_position_nocheck for an offloaded convertor.  The
 * device program resumes at any byte from bConverted alone, so the
 * reference's stack (pStack / stack_pos / partial_length: the host walk's
 * state) is not needed: a receive goes to exactly `*position` (a partial
 * element is unpacked byte for byte); a send of a non-contiguous type
 * moves back to the start of the predefined element holding it, as the
 * reference does (opal_convertor.c:433-443: "don't allow it to move in the
 * middle of a predefined datatype"). */
int32_t opal_rocm_set_position(opal_convertor_t *convertor, size_t *position)
{
    const opal_datatype_t *dt = convertor->pDesc;
    size_t pos = *position;
    if ((convertor->flags & CONVERTOR_SEND) && !(dt->flags & OPAL_DATATYPE_FLAG_CONTIGUOUS) &&
        dt->size > 0) {
        const size_t inst = pos / dt->size;
        pos = inst * dt->size +
              snap_in(dt->opt_desc.desc, 0, (uint32_t)dt->opt_desc.used, pos - inst * dt->size, 0);
    }
    convertor->bConverted = pos;
    convertor->partial_length = 0;
    *position = pos;
    return 0;
}
