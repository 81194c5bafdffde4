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

/* ------------------------------------------------ per-convertor state */

/* What a conversion carries between fAdvance calls (opal_convertor_t has no
 * field for it): kept beside the convertor, keyed by its address, reset at
 * every prepare (select) and released when the conversion completes.
 *
 *  - deferred device fragments (a caller that asked for it with
 *    opal_rocm_set_copy_function_async): fAdvance records the iovecs and
 *    returns; the next flush (opal_rocm_record_event, a synchronous call,
 *    a set_position) launches one kernel over all of them.  One fAdvance
 *    per 64 KiB fragment then costs a few host instructions, and a train
 *    of fragments one launch (the reference pays a cuMemcpy per run per
 *    fragment, opal_datatype_cuda.c:121-145).
 *  - host fragments (btl/sm's shared-memory fragments, MPI_Pack into host
 *    memory): the device never touches a host iovec — that memory is not
 *    mapped for it.  A send packs a window of up to WIN_BYTES of the stream
 *    ahead with one launch, copies it to page-locked memory once, and
 *    serves that fragment and the following ones from there with memcpy; a
 *    receive gathers host fragments in page-locked memory and unpacks a
 *    window at a time (at the latest when the stream completes). */
#define WIN_BYTES ((size_t) 16 << 20)

typedef struct {
    const opal_convertor_t *conv;
    void *stream;   /* async stream (ROCm-only build: the convertor has no field) */
    int defer;      /* device fragments are recorded, launched at the next flush */
    struct iovec *dq;
    uint32_t ndq, capdq;
    size_t dq_pos, dq_end;  /* stream range of the recorded fragments */
    char *win_dev, *win_host;
    size_t win_pos, win_end;  /* stream range held in win_host */
    uintptr_t dev_lo, dev_hi; /* the device allocation the last fragment was in */
} conv_state;

static conv_state **g_states;
static int g_nstates, g_capstates;
static pthread_mutex_t g_state_lock = PTHREAD_MUTEX_INITIALIZER;
/* released windows, reused (page-locked allocations are slow to make) */
#define WIN_POOL 4
static char *g_pool_dev[WIN_POOL], *g_pool_host[WIN_POOL];
static int g_npool;

/* the last state this thread used, valid while no state was dropped since
 * (g_epoch): the per-fragment lookup without the lock */
static unsigned long g_epoch;
static __thread conv_state *tl_state;
static __thread unsigned long tl_epoch;

static conv_state *state_of(const opal_convertor_t *c, int create)
{
    conv_state *st = NULL;
    if (tl_state && tl_state->conv == c && tl_epoch == __atomic_load_n(&g_epoch, __ATOMIC_ACQUIRE))
        return tl_state;
    pthread_mutex_lock(&g_state_lock);
    for (int i = 0; i < g_nstates; ++i)
        if (g_states[i]->conv == c) {
            st = g_states[i];
            break;
        }
    if (!st && create) {
        if (g_nstates == g_capstates) {
            const int cap = g_capstates ? 2 * g_capstates : 16;
            conv_state **n = realloc(g_states, (size_t) cap * sizeof(*n));
            if (n) {
                g_states = n;
                g_capstates = cap;
            }
        }
        if (g_nstates < g_capstates && (st = calloc(1, sizeof(*st)))) {
            st->conv = c;
            g_states[g_nstates++] = st;
        }
    }
    if (st) {
        tl_state = st;
        tl_epoch = __atomic_load_n(&g_epoch, __ATOMIC_ACQUIRE);
    }
    pthread_mutex_unlock(&g_state_lock);
    return st;
}

static void state_drop(const opal_convertor_t *c)
{
    conv_state *st = NULL;
    pthread_mutex_lock(&g_state_lock);
    for (int i = 0; i < g_nstates; ++i)
        if (g_states[i]->conv == c) {
            st = g_states[i];
            g_states[i] = g_states[--g_nstates];
            __atomic_add_fetch(&g_epoch, 1, __ATOMIC_RELEASE);  /* every thread's cache */
            break;
        }
    if (st && st->win_dev) {
        if (g_npool < WIN_POOL) {
            g_pool_dev[g_npool] = st->win_dev;
            g_pool_host[g_npool++] = st->win_host;
            st->win_dev = st->win_host = NULL;
        }
    }
    pthread_mutex_unlock(&g_state_lock);
    if (!st) return;
    (void) ompi_amd_device_free(st->win_dev);
    (void) ompi_amd_host_free(st->win_host);
    free(st->dq);
    free(st);
}

static int state_window(conv_state *st)
{
    if (st->win_dev) return 0;
    pthread_mutex_lock(&g_state_lock);
    if (g_npool > 0) {
        st->win_dev = g_pool_dev[--g_npool];
        st->win_host = g_pool_host[g_npool];
    }
    pthread_mutex_unlock(&g_state_lock);
    if (st->win_dev) return 0;
    if (0 != ompi_amd_device_alloc((void **) &st->win_dev, WIN_BYTES) ||
        0 != ompi_amd_host_alloc((void **) &st->win_host, WIN_BYTES)) {
        (void) ompi_amd_device_free(st->win_dev);
        st->win_dev = NULL;
        return -1;
    }
    return 0;
}

static void *stream_of(const opal_convertor_t *c, const conv_state *st)
{
    return NULL != st && NULL != st->stream ? st->stream : conv_stream(c);
}

/* launch the recorded device fragments (one kernel over all of them) */
static int flush_dq(opal_convertor_t *c, conv_state *st, ompi_amd_ddt_t *prog, int unpack)
{
    if (!st || 0 == st->ndq) return 0;
    uint32_t n = st->ndq;
    size_t moved = 0;
    const int rc = unpack
        ? ompi_amd_ddt_unpack_iov(prog, c->count, c->pBaseBuf, st->dq_pos,
                                  (ompi_amd_iovec_t *) st->dq, &n, &moved, stream_of(c, st))
        : ompi_amd_ddt_pack_iov(prog, c->count, c->pBaseBuf, st->dq_pos,
                                (ompi_amd_iovec_t *) st->dq, &n, &moved, stream_of(c, st));
    st->ndq = 0;
    return rc < 0 || moved != st->dq_end - st->dq_pos ? -1 : 0;
}

/* a receive's gathered host window onto the device, unpacked (and waited
 * for: the window is refilled only after the device read it) */
static int flush_win(opal_convertor_t *c, conv_state *st, ompi_amd_ddt_t *prog)
{
    if (!st || st->win_end == st->win_pos) return 0;
    const size_t n = st->win_end - st->win_pos;
    void *s = stream_of(c, st);
    struct iovec v = {st->win_dev, n};
    uint32_t one = 1;
    size_t moved = 0;
    int rc = ompi_amd_memcpy_async(st->win_dev, st->win_host, n, s);
    if (0 == rc)
        rc = ompi_amd_ddt_unpack_iov(prog, c->count, c->pBaseBuf, st->win_pos,
                                     (ompi_amd_iovec_t *) &v, &one, &moved, s) < 0 ? -1 : 0;
    if (0 == rc) rc = ompi_amd_stream_synchronize(s);
    st->win_pos = st->win_end;
    return 0 == rc && moved == n ? 0 : -1;
}

/* a send's window [pos, pos + n) packed on the device and copied to host */
static int fill_win(opal_convertor_t *c, conv_state *st, ompi_amd_ddt_t *prog, size_t pos, size_t n)
{
    void *s = stream_of(c, st);
    struct iovec v = {st->win_dev, n};
    uint32_t one = 1;
    size_t moved = 0;
    if (ompi_amd_ddt_pack_iov(prog, c->count, c->pBaseBuf, pos, (ompi_amd_iovec_t *) &v, &one,
                              &moved, s) < 0 || moved != n ||
        0 != ompi_amd_memcpy_async(st->win_host, st->win_dev, n, s) ||
        0 != ompi_amd_stream_synchronize(s)) {
        st->win_pos = st->win_end = 0;
        return -1;
    }
    st->win_pos = pos;
    st->win_end = pos + n;
    return 0;
}

/* a fragment in device memory?  The allocation of the previous one is
 * remembered, so a train of fragments in one buffer asks the runtime once */
static int on_device(conv_state *st, const void *p)
{
    void *b = NULL;
    size_t n = 0;
    if ((uintptr_t) p >= st->dev_lo && (uintptr_t) p < st->dev_hi) return 1;
    if (1 != ompi_amd_pointer_range(p, &b, &n)) return 0;
    st->dev_lo = (uintptr_t) b;
    st->dev_hi = (uintptr_t) b + n;
    return 1;
}

static int record_dq(conv_state *st, void *base, size_t len, size_t pos)
{
    if (st->ndq == st->capdq) {
        const uint32_t cap = st->capdq ? 2 * st->capdq : 64;
        struct iovec *n = realloc(st->dq, (size_t) cap * sizeof(*n));
        if (!n) return -1;
        st->dq = n;
        st->capdq = cap;
    }
    if (0 == st->ndq) st->dq_pos = pos;
    st->dq[st->ndq].iov_base = base;
    st->dq[st->ndq++].iov_len = len;
    st->dq_end = pos + len;
    return 0;
}

/* ------------------------------------------------------ advance step */

static int32_t advance(opal_convertor_t *conv, struct iovec *iov, uint32_t *out_size,
                       size_t *max_data, int unpack)
{
    ompi_amd_ddt_t *prog = program_of(conv->pDesc, 0);
    if (!prog) return -1;
    const size_t total = ompi_amd_ddt_size(prog) * conv->count;
    size_t pos = conv->bConverted;
    uint32_t used = 0;
    conv_state *st = state_of(conv, 1);
    if (!st) return -1;
    const int defer = st->defer;
    int direct = 0;  /* device fragments of this call not recorded: launched now */
    *max_data = 0;
    for (uint32_t i = 0; i < *out_size && pos < total; ++i) {
        const size_t take = iov[i].iov_len < total - pos ? iov[i].iov_len : total - pos;
        iov[i].iov_len = take;
        used = i + 1;
        if (0 == take) continue;
        if (NULL == iov[i].iov_base) return -1;
        if (on_device(st, iov[i].iov_base)) {
            if (st->ndq && st->dq_end != pos && 0 != flush_dq(conv, st, prog, unpack)) return -1;
            if (0 != record_dq(st, iov[i].iov_base, take, pos)) return -1;
            direct = !defer;
        } else {  /* a host fragment: through the page-locked window */
            if (0 != state_window(st)) return -1;
            for (size_t done = 0; done < take;) {
                const size_t at = pos + done;
                if (!unpack) {
                    if (at < st->win_pos || at >= st->win_end) {
                        const size_t n = total - at < WIN_BYTES ? total - at : WIN_BYTES;
                        if (0 != fill_win(conv, st, prog, at, n)) return -1;
                    }
                    size_t m = st->win_end - at;
                    if (m > take - done) m = take - done;
                    memcpy((char *) iov[i].iov_base + done, st->win_host + (at - st->win_pos), m);
                    done += m;
                } else {
                    if (st->win_end != at || st->win_end - st->win_pos == WIN_BYTES) {
                        if (0 != flush_win(conv, st, prog)) return -1;
                        st->win_pos = st->win_end = at;
                    }
                    size_t m = WIN_BYTES - (st->win_end - st->win_pos);
                    if (m > take - done) m = take - done;
                    memcpy(st->win_host + (st->win_end - st->win_pos), (char *) iov[i].iov_base + done, m);
                    st->win_end += m;
                    done += m;
                }
            }
        }
        pos += take;
    }
    if (pos < total) used = *out_size;
    *out_size = used;
    *max_data = pos - conv->bConverted;
    conv->bConverted = pos;
    const int complete = pos == total;
    if ((direct || (complete && !defer)) && 0 != flush_dq(conv, st, prog, unpack)) return -1;
    if (unpack && complete && 0 != flush_win(conv, st, prog)) return -1;
    /* a launch of this call: synchronous unless the caller runs the
     * convertor asynchronously and waits on its stream itself
     * (CONVERTOR_CUDA_ASYNC: opal_cuda_set_copy_function_async in a CUDA
     * build, opal_rocm_set_copy_function_async here) */
    if (direct && !(conv->flags & CONVERTOR_CUDA_ASYNC) &&
        0 != ompi_amd_stream_synchronize(stream_of(conv, st)))
        return -1;
    if (complete) {
        conv->flags |= CONVERTOR_COMPLETED;
        if (!defer) state_drop(conv);
    }
    return complete ? 1 : 0;
}

/* A whole typed buffer to / from a packed device buffer in one launch
 * (pml/rocm's non-contiguous device messages) */
static int whole(const opal_datatype_t *dt, size_t count, void *typed, void *packed, void *stream,
                 int unpack)
{
    ompi_amd_ddt_t *prog;
    if (0 == count || 0 == dt->size) return 0;
    if (!ompi_amd_is_device_pointer((const char *) typed + dt->true_lb) ||
        !ompi_amd_is_device_pointer(packed) || !(prog = program_of(dt, 1)))
        return 1;
    size_t done = 0;
    const int rc = unpack
        ? ompi_amd_ddt_unpack(prog, count, packed, typed, 0, dt->size * count, &done, stream)
        : ompi_amd_ddt_pack(prog, count, typed, packed, 0, dt->size * count, &done, stream);
    if (rc < 0 || done != dt->size * count || 0 != ompi_amd_stream_synchronize(stream)) return -1;
    return 0;
}

int opal_rocm_device_program(const opal_datatype_t *dt)
{
    return NULL != program_of(dt, 1);
}

const ompi_amd_ddt_t *opal_rocm_device_ddt(const opal_datatype_t *dt)
{
    return program_of(dt, 1);
}

int opal_rocm_pack_device(const opal_datatype_t *dt, size_t count, const void *src, void *packed,
                          void *stream)
{
    return whole(dt, count, (void *) src, packed, stream, 0);
}

int opal_rocm_unpack_device(const opal_datatype_t *dt, size_t count, const void *packed, void *dst,
                            void *stream)
{
    return whole(dt, count, dst, (void *) packed, stream, 1);
}

int opal_rocm_set_copy_function_async(opal_convertor_t *convertor, void *stream)
{
    conv_state *st = state_of(convertor, 1);
    if (!st) return -1;
    convertor->flags |= CONVERTOR_CUDA_ASYNC;
#if OPAL_CUDA_SUPPORT
    convertor->stream = stream;
#endif
    st->stream = stream;
    st->defer = 1;
    return 0;
}

int opal_rocm_convertor_flush(opal_convertor_t *convertor)
{
    conv_state *st = state_of(convertor, 0);
    ompi_amd_ddt_t *prog;
    if (!st) return 0;
    if (!(prog = program_of(convertor->pDesc, 0))) return -1;
    const int unpack = !(convertor->flags & CONVERTOR_SEND);
    if (0 != flush_dq(convertor, st, prog, unpack)) return -1;
    if (unpack && 0 != flush_win(convertor, st, prog)) return -1;
    return 0;
}

int opal_rocm_record_event(opal_convertor_t *convertor, void **event)
{
    conv_state *st = state_of(convertor, 0);
    if (0 != opal_rocm_convertor_flush(convertor)) return -1;
    return 0 == ompi_amd_event_record(event, stream_of(convertor, st)) ? 0 : -1;
}

void opal_rocm_convertor_release(opal_convertor_t *convertor)
{
    state_drop(convertor);
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
    if (g_nstates) state_drop(convertor);  /* a new conversion at this address */
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
    /* recorded fragments and a gathered window belong to the old position */
    if (0 != opal_rocm_convertor_flush(convertor)) return -1;
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
