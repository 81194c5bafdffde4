/*
 * TEST HARNESS ONLY: drives the convertor seam (ompi_amd/mca/common/rocm)
 * through a minimal stand-in of opal's convertor entry points, the way a
 * PML drives opal_convertor_pack / _unpack with fragment-sized iovecs, and
 * checks every byte against the oracle (oracle/ddt_oracle.c).
 *
 * Input on stdin, one datatype per block (written by tests/test_mca_glue.py
 * from tests/golden/ddt_kat.json plus loop-shaped descriptions):
 *   T <name> <count> <extent> <size>
 *   B <nblocks> <disp len>...            the typemap runs (oracle)
 *   D <ndesc>, then per entry one of     the opt_desc description:
 *     E <type> <count> <blocklen> <extent> <disp>
 *     L <items> <loops> <extent>
 *     X <items> <size>
 *   C <nchunks> <chunk>...               fragment sizes
 * HARNESS_GPU=0: only the table / selection checks that need no GPU.
 */
#include <stdint.h>
#include <stdio.h>
#include <stdlib.h>
#include <string.h>

#include "opal/datatype/opal_convertor.h"
#include "opal/datatype/opal_datatype.h"
#if OPAL_CUDA_SUPPORT
#include "opal/datatype/opal_datatype_cuda.h"
#endif
#include "opal/datatype/opal_datatype_internal.h"

#include "../../oracle/oracle.h"
#include "ompi_amd.h"
#include "opal_datatype_rocm.h"

int harness_dev_alloc_copy(void **d, const void *h, size_t bytes);
int harness_dev_copy_in(void *d, const void *h, size_t bytes);
int harness_dev_copy_back(void *h, const void *d, size_t bytes);
int harness_dev_free(void *d);

/* ---- stand-ins of what opal itself provides ---- */
static opal_datatype_t basic[OPAL_DATATYPE_MAX_PREDEFINED];
const opal_datatype_t *opal_datatype_basicDatatypes[OPAL_DATATYPE_MAX_PREDEFINED];

static int gpu_enabled;
#if OPAL_CUDA_SUPPORT
static opal_common_cuda_function_table_t ftable;

void opal_cuda_add_initialization_function(int (*fptr)(opal_common_cuda_function_table_t *))
{
    gpu_enabled = fptr(&ftable) == 0;
}

/* mca_cuda_convertor_init (opal_datatype_cuda.c:44-60), restated */
void mca_cuda_convertor_init(opal_convertor_t *convertor, const void *pUserBuf)
{
    if (gpu_enabled && ftable.gpu_is_gpu_buffer(pUserBuf, convertor)) convertor->flags |= CONVERTOR_CUDA;
}
#endif

/* prepare_for_send / _recv reduced to what this test needs: homogeneous,
 * non-contiguous; then the two lines INTEGRATION.md §3 adds to the
 * reference's prepare functions (offload the advance function). */
static int32_t prepare(opal_convertor_t *c, const opal_datatype_t *dt, size_t count, const void *buf,
                       uint32_t dir)
{
    memset(c, 0, sizeof(*c));
    c->flags = dir | CONVERTOR_HOMOGENEOUS;
#if OPAL_CUDA_SUPPORT
    mca_cuda_convertor_init(c, buf);
#endif
    c->local_size = count * dt->size;
    c->pBaseBuf = (unsigned char *)buf;
    c->count = count;
    c->pDesc = dt;
    c->use_desc = &dt->opt_desc;
    c->pStack = c->static_stack;
    c->stack_size = DT_STATIC_STACK_SIZE;
    c->fAdvance = NULL;  /* the reference's generic functions are not built here */
    if (count == 0 || dt->size == 0) c->flags |= CONVERTOR_COMPLETED;
    opal_rocm_convertor_select(c);
    return 0;
}

/* opal_convertor_set_position (opal_convertor.h:313-346) restated; the
 * nocheck step of an offloaded convertor is the seam's hook */
int32_t opal_convertor_set_position(opal_convertor_t *c, size_t *position)
{
    if (c->local_size <= *position) {
        c->flags |= CONVERTOR_COMPLETED;
        c->bConverted = c->local_size;
        *position = c->bConverted;
        return 0;
    }
    if (*position == c->bConverted) return 0;
    c->flags &= ~CONVERTOR_COMPLETED;
    if (!opal_rocm_convertor_owns(c)) return -1;  /* the host walk is not built here */
    return opal_rocm_set_position(c, position);
}

int32_t opal_convertor_prepare_for_send(opal_convertor_t *c, const struct opal_datatype_t *dt,
                                        size_t count, const void *buf)
{
    return prepare(c, dt, count, buf, CONVERTOR_SEND);
}

int32_t opal_convertor_prepare_for_recv(opal_convertor_t *c, const struct opal_datatype_t *dt,
                                        size_t count, const void *buf)
{
    return prepare(c, dt, count, buf, CONVERTOR_RECV);
}

/* opal_convertor_pack / _unpack (opal_convertor.c:218-325) for the
 * non-NO_OP case: the completed guard, then fAdvance */
static int32_t run(opal_convertor_t *c, struct iovec *iov, uint32_t *out, size_t *max)
{
    if (c->flags & CONVERTOR_COMPLETED) {
        iov[0].iov_len = 0;
        *out = 0;
        *max = 0;
        return 1;
    }
    if (!c->fAdvance) return -1;
    return c->fAdvance(c, iov, out, max);
}

int32_t opal_convertor_pack(opal_convertor_t *c, struct iovec *iov, uint32_t *out, size_t *max)
{
    return run(c, iov, out, max);
}

int32_t opal_convertor_unpack(opal_convertor_t *c, struct iovec *iov, uint32_t *out, size_t *max)
{
    return run(c, iov, out, max);
}

/* ---- the test ---- */
typedef struct {
    char kind;  /* 'T' fragment trains, 'U' out-of-order unpack, 'P' position.c replay */
    char name[64];
    size_t count;
    int64_t extent;
    size_t size;
    int nb;
    orc_block_t *blocks;
    int nd;
    dt_elem_desc_t *desc;
    int nchunks;
    size_t chunks[16];
    int nfrag;                /* U: the fragment table (bytes, offset) */
    size_t frags[32][2];
    unsigned char *init, *packed, *expect;  /* U: typed initial, packed stream, typed expected */
    size_t ninit, npacked, nexpect;
    size_t seg;               /* P: segment length */
} spec_t;

static int read_hex(FILE *f, unsigned char **out, size_t *n)
{
    size_t len = 0;
    if (fscanf(f, "%zu", &len) != 1) return -1;
    unsigned char *b = malloc(len + 1);
    for (size_t i = 0; i < len; ++i) {
        unsigned v;
        if (fscanf(f, "%2x", &v) != 1) {
            free(b);
            return -1;
        }
        b[i] = (unsigned char) v;
    }
    *out = b;
    *n = len;
    return 0;
}

static uint64_t rng_state = 0x9e3779b97f4a7c15ull;
static uint8_t rnd8(void)
{
    rng_state ^= rng_state >> 12;
    rng_state ^= rng_state << 25;
    rng_state ^= rng_state >> 27;
    return (uint8_t)((rng_state * 0x2545f4914f6cdd1dull) >> 56);
}

static int read_spec(FILE *f, spec_t *s)
{
    char tag[4];
    memset(s, 0, sizeof(*s));
    if (fscanf(f, "%3s", tag) != 1) return 0;
    if ((strcmp(tag, "T") && strcmp(tag, "U") && strcmp(tag, "P")) ||
        fscanf(f, "%63s %zu %ld %zu", s->name, &s->count, &s->extent, &s->size) != 4)
        return -1;
    s->kind = tag[0];
    if (fscanf(f, "%3s %d", tag, &s->nb) != 2 || strcmp(tag, "B")) return -1;
    s->blocks = calloc((size_t)s->nb, sizeof(orc_block_t));
    for (int i = 0; i < s->nb; ++i)
        if (fscanf(f, "%ld %ld", &s->blocks[i].disp, &s->blocks[i].len) != 2) return -1;
    if (fscanf(f, "%3s %d", tag, &s->nd) != 2 || strcmp(tag, "D")) return -1;
    s->desc = calloc((size_t)s->nd, sizeof(dt_elem_desc_t));
    for (int i = 0; i < s->nd; ++i) {
        dt_elem_desc_t *d = &s->desc[i];
        if (fscanf(f, "%3s", tag) != 1) return -1;
        if (!strcmp(tag, "E")) {
            unsigned type, count;
            size_t bl;
            long ext, disp;
            if (fscanf(f, "%u %u %zu %ld %ld", &type, &count, &bl, &ext, &disp) != 5) return -1;
            d->elem.common.type = (uint16_t)type;
            d->elem.common.flags = OPAL_DATATYPE_FLAG_DATA;
            d->elem.count = count;
            d->elem.blocklen = bl;
            d->elem.extent = ext;
            d->elem.disp = disp;
        } else if (!strcmp(tag, "L")) {
            unsigned items, loops;
            long ext;
            if (fscanf(f, "%u %u %ld", &items, &loops, &ext) != 3) return -1;
            d->loop.common.type = OPAL_DATATYPE_LOOP;
            d->loop.items = items;
            d->loop.loops = loops;
            d->loop.extent = ext;
        } else if (!strcmp(tag, "X")) {
            unsigned items;
            size_t size;
            if (fscanf(f, "%u %zu", &items, &size) != 2) return -1;
            d->end_loop.common.type = OPAL_DATATYPE_END_LOOP;
            d->end_loop.items = items;
            d->end_loop.size = size;
        } else {
            return -1;
        }
    }
    if (s->kind == 'U') {
        if (fscanf(f, "%3s %d", tag, &s->nfrag) != 2 || strcmp(tag, "F") || s->nfrag > 32) return -1;
        for (int i = 0; i < s->nfrag; ++i)
            if (fscanf(f, "%zu %zu", &s->frags[i][0], &s->frags[i][1]) != 2) return -1;
        if (fscanf(f, "%3s", tag) != 1 || strcmp(tag, "I") || read_hex(f, &s->init, &s->ninit)) return -1;
        if (fscanf(f, "%3s", tag) != 1 || strcmp(tag, "P") || read_hex(f, &s->packed, &s->npacked)) return -1;
        if (fscanf(f, "%3s", tag) != 1 || strcmp(tag, "E") || read_hex(f, &s->expect, &s->nexpect)) return -1;
        return 1;
    }
    if (s->kind == 'P') {
        if (fscanf(f, "%3s %zu", tag, &s->seg) != 2 || strcmp(tag, "S") || s->seg == 0) return -1;
        return 1;
    }
    if (fscanf(f, "%3s %d", tag, &s->nchunks) != 2 || strcmp(tag, "C") || s->nchunks > 16) return -1;
    for (int i = 0; i < s->nchunks; ++i)
        if (fscanf(f, "%zu", &s->chunks[i]) != 1) return -1;
    return 1;
}

/* Drive a whole stream through the convertor in calls of `niov` entries of
 * `chunk` bytes (the PML's fragment train); contig is the packed buffer on
 * the device.  Returns 0 on success. */
static int drive(opal_convertor_t *c, char *contig, size_t total, size_t chunk, uint32_t niov,
                 int unpack, char *why, size_t whylen)
{
    size_t pos = 0;
    struct iovec iov[8];
    for (int calls = 0;; ++calls) {
        if (calls > 4000000) {
            snprintf(why, whylen, "no progress at %zu", pos);
            return -1;
        }
        size_t room = 0;
        for (uint32_t k = 0; k < niov; ++k) {
            iov[k].iov_base = contig + pos + room;
            iov[k].iov_len = chunk;
            room += chunk;
        }
        uint32_t out = niov;
        size_t max = room;
        const int32_t rc = unpack ? opal_convertor_unpack(c, iov, &out, &max)
                                  : opal_convertor_pack(c, iov, &out, &max);
        if (rc < 0) {
            snprintf(why, whylen, "advance returned %d at %zu: %s", rc, pos, ompi_amd_last_error());
            return -1;
        }
        size_t sum = 0;
        for (uint32_t k = 0; k < out; ++k) sum += iov[k].iov_len;
        if (sum != max || out > niov || c->bConverted != pos + max) {
            snprintf(why, whylen, "contract: out %u sum %zu max %zu bConverted %zu pos %zu", out, sum,
                     max, c->bConverted, pos);
            return -1;
        }
        pos += max;
        if (rc == 1) break;
        if (max != room) {
            snprintf(why, whylen, "short call (%zu of %zu) without completion", max, room);
            return -1;
        }
    }
    if (pos != total) {
        snprintf(why, whylen, "stream ended at %zu of %zu", pos, total);
        return -1;
    }
    return 0;
}

static int test_type(const spec_t *s)
{
    opal_datatype_t dt;
    memset(&dt, 0, sizeof(dt));
    dt.size = s->size;
    dt.lb = 0;
    dt.ub = s->extent;
    dt.opt_desc.length = dt.opt_desc.used = (size_t)s->nd;
    dt.opt_desc.desc = s->desc;
    const size_t total = s->size * s->count, tbytes = (size_t)s->extent * s->count + 64;
    char *typed = malloc(tbytes), *exp = malloc(total + 64), *got = malloc(total + 64);
    char *bg = malloc(tbytes), *texp = malloc(tbytes), *tgot = malloc(tbytes);
    for (size_t i = 0; i < tbytes; ++i) typed[i] = (char)rnd8();
    for (size_t i = 0; i < tbytes; ++i) bg[i] = (char)rnd8();
    orc_pack(s->blocks, s->nb, s->extent, s->count, typed, exp, 0, total);
    memcpy(texp, bg, tbytes);
    orc_unpack(s->blocks, s->nb, s->extent, s->count, exp, texp, 0, total);
    void *dtyped = NULL, *dpack = NULL, *dexp = NULL, *dtyped2 = NULL;
    int fails = 0;
    char why[256] = "";
    if (harness_dev_alloc_copy(&dtyped, typed, tbytes) || harness_dev_alloc_copy(&dpack, got, total + 64) ||
        harness_dev_alloc_copy(&dexp, exp, total + 64) || harness_dev_alloc_copy(&dtyped2, bg, tbytes)) {
        printf("FAIL %s: device allocation\n", s->name);
        return 1;
    }
    for (int ci = 0; ci < s->nchunks; ++ci) {
        for (uint32_t niov = 1; niov <= 7; niov += 6) {
            opal_convertor_t c;
            /* pack */
            opal_convertor_prepare_for_send(&c, &dt, s->count, dtyped);
            if (c.fAdvance != opal_rocm_pack) {
                printf("FAIL %s: pack not offloaded (flags %x)\n", s->name, c.flags);
                ++fails;
                continue;
            }
            if (drive(&c, dpack, total, s->chunks[ci], niov, 0, why, sizeof(why)) ||
                harness_dev_copy_back(got, dpack, total) || memcmp(got, exp, total)) {
                size_t bad = 0;
                while (bad < total && got[bad] == exp[bad]) ++bad;
                printf("FAIL %s pack chunk %zu x%u: %s (first byte differing %zu)\n", s->name,
                       s->chunks[ci], niov, why, bad);
                ++fails;
            }
            /* unpack into a buffer whose gaps must survive */
            harness_dev_copy_in(dtyped2, bg, tbytes);
            opal_convertor_prepare_for_recv(&c, &dt, s->count, dtyped2);
            if (c.fAdvance != opal_rocm_unpack) {
                printf("FAIL %s: unpack not offloaded\n", s->name);
                ++fails;
                continue;
            }
            if (drive(&c, dexp, total, s->chunks[ci], niov, 1, why, sizeof(why)) ||
                harness_dev_copy_back(tgot, dtyped2, tbytes) || memcmp(tgot, texp, tbytes)) {
                size_t bad = 0;
                while (bad < tbytes && tgot[bad] == texp[bad]) ++bad;
                printf("FAIL %s unpack chunk %zu x%u: %s (first byte differing %zu)\n", s->name,
                       s->chunks[ci], niov, why, bad);
                ++fails;
            }
            /* host fragments (btl/sm's shared-memory fragments): the
             * page-locked windows, never a kernel on host memory */
            memset(got, 0, total);
            opal_convertor_prepare_for_send(&c, &dt, s->count, dtyped);
            if (drive(&c, got, total, s->chunks[ci], niov, 0, why, sizeof(why)) || memcmp(got, exp, total)) {
                printf("FAIL %s pack into host fragments, chunk %zu x%u: %s\n", s->name, s->chunks[ci],
                       niov, why);
                ++fails;
            }
            harness_dev_copy_in(dtyped2, bg, tbytes);
            opal_convertor_prepare_for_recv(&c, &dt, s->count, dtyped2);
            if (drive(&c, exp, total, s->chunks[ci], niov, 1, why, sizeof(why)) ||
                harness_dev_copy_back(tgot, dtyped2, tbytes) || memcmp(tgot, texp, tbytes)) {
                printf("FAIL %s unpack from host fragments, chunk %zu x%u: %s\n", s->name,
                       s->chunks[ci], niov, why);
                ++fails;
            }
            /* asynchronous conversion: device fragments recorded, one launch
             * at the event (opal_rocm_set_copy_function_async / _record_event) */
            for (int dir = 0; dir < 2; ++dir) {
                void *ev = NULL;
                harness_dev_copy_in(dtyped2, bg, tbytes);
                harness_dev_copy_in(dpack, bg, total);
                if (dir == 0) opal_convertor_prepare_for_send(&c, &dt, s->count, dtyped);
                else opal_convertor_prepare_for_recv(&c, &dt, s->count, dtyped2);
                if (opal_rocm_set_copy_function_async(&c, NULL) != 0 ||
                    drive(&c, dir == 0 ? dpack : dexp, total, s->chunks[ci], niov, dir, why, sizeof(why)) ||
                    opal_rocm_record_event(&c, &ev) != 0 || ompi_amd_event_synchronize(ev) != 0) {
                    printf("FAIL %s deferred %s chunk %zu x%u: %s\n", s->name, dir ? "unpack" : "pack",
                           s->chunks[ci], niov, why);
                    ++fails;
                } else if (dir == 0 ? (harness_dev_copy_back(got, dpack, total) || memcmp(got, exp, total))
                                    : (harness_dev_copy_back(tgot, dtyped2, tbytes) ||
                                       memcmp(tgot, texp, tbytes))) {
                    printf("FAIL %s deferred %s chunk %zu x%u: bytes differ\n", s->name,
                           dir ? "unpack" : "pack", s->chunks[ci], niov);
                    ++fails;
                }
                ompi_amd_event_destroy(ev);
                opal_rocm_convertor_release(&c);
            }
        }
    }
    harness_dev_free(dtyped);
    harness_dev_free(dpack);
    harness_dev_free(dexp);
    harness_dev_free(dtyped2);
    free(typed); free(exp); free(got); free(bg); free(texp); free(tgot);
    if (!fails) printf("ok %s\n", s->name);
    return fails;
}

static void type_of_spec(const spec_t *s, opal_datatype_t *dt)
{
    memset(dt, 0, sizeof(*dt));
    dt->size = s->size;
    dt->lb = dt->true_lb = 0;
    dt->ub = dt->true_ub = s->extent;
    dt->opt_desc.length = dt->opt_desc.used = (size_t)s->nd;
    dt->opt_desc.desc = s->desc;
}

/* unpack_ooo.c:75-131: a receive convertor over the typed buffer; every
 * fragment (bytes, offset) of the table unpacked after set_position, out of
 * order; the whole typed buffer must equal the expected bytes */
static int test_unpack_ooo(const spec_t *s)
{
    opal_datatype_t dt;
    opal_convertor_t c;
    void *dtyped = NULL, *dpacked = NULL;
    unsigned char *got = malloc(s->ninit);
    int fails = 0;
    type_of_spec(s, &dt);
    if (s->ninit != s->nexpect || s->npacked != s->size * s->count ||
        harness_dev_alloc_copy(&dtyped, s->init, s->ninit) ||
        harness_dev_alloc_copy(&dpacked, s->packed, s->npacked)) {
        printf("FAIL %s: fixture sizes / device allocation\n", s->name);
        return 1;
    }
    opal_convertor_prepare_for_recv(&c, &dt, s->count, dtyped);
    if (c.fAdvance != opal_rocm_unpack) {
        printf("FAIL %s: unpack not offloaded (flags %x)\n", s->name, c.flags);
        return 1;
    }
    for (int i = 0; i < s->nfrag && !fails; ++i) {
        size_t pos = s->frags[i][1], max = s->frags[i][0];
        struct iovec iov = {(char *) dpacked + s->frags[i][1], s->frags[i][0]};
        uint32_t n = 1;
        opal_convertor_set_position(&c, &pos);
        if (pos != s->frags[i][1]) {
            printf("FAIL %s: set_position(%zu) gave %zu\n", s->name, s->frags[i][1], pos);
            ++fails;
            break;
        }
        const int32_t rc = opal_convertor_unpack(&c, &iov, &n, &max);
        if (rc < 0 || max != s->frags[i][0] || c.bConverted != s->frags[i][1] + s->frags[i][0]) {
            printf("FAIL %s: fragment %d (%zu at %zu): rc %d max %zu bConverted %zu: %s\n", s->name, i,
                   s->frags[i][0], s->frags[i][1], rc, max, c.bConverted, ompi_amd_last_error());
            ++fails;
        }
    }
    if (!fails && (harness_dev_copy_back(got, dtyped, s->ninit) || memcmp(got, s->expect, s->ninit))) {
        size_t bad = 0;
        while (bad < s->ninit && got[bad] == s->expect[bad]) ++bad;
        printf("FAIL %s: typed buffer differs from the expected at byte %zu (element %zu, offset %zu)\n",
               s->name, bad, bad / (size_t) s->extent, bad % (size_t) s->extent);
        ++fails;
    }
    harness_dev_free(dtyped);
    harness_dev_free(dpacked);
    free(got);
    if (!fails) printf("ok %s\n", s->name);
    return fails;
}

/* position.c:90-250 replayed on device buffers: create_segments (a send
 * convertor's set_position finds each segment's end), shuffle_segments
 * (every other pair from the ends swapped), pack_segments and
 * unpack_segments in that order; packed segments must equal the oracle's
 * stream at their positions and the received typed buffer the sent one
 * (gaps untouched) */
static int test_position(const spec_t *s)
{
    opal_datatype_t dt;
    opal_convertor_t c;
    const size_t total = s->size * s->count, tbytes = (size_t) s->extent * s->count;
    size_t nseg = 0, pos = 0;
    size_t (*segs)[2] = malloc(sizeof(*segs) * (total + 1));
    char *typed = malloc(tbytes), *bg = malloc(tbytes), *stream = malloc(total), *got = malloc(tbytes);
    char *exp = malloc(tbytes), *pk = malloc(total);
    void *dsend = NULL, *drecv = NULL, *dseg = NULL;
    int fails = 0;
    type_of_spec(s, &dt);
    for (size_t i = 0; i < tbytes; ++i) typed[i] = (char) rnd8();
    for (size_t i = 0; i < tbytes; ++i) bg[i] = (char) rnd8();
    orc_pack(s->blocks, s->nb, s->extent, s->count, typed, stream, 0, total);
    memcpy(exp, bg, tbytes);
    orc_unpack(s->blocks, s->nb, s->extent, s->count, stream, exp, 0, total);
    if (harness_dev_alloc_copy(&dsend, typed, tbytes) || harness_dev_alloc_copy(&drecv, bg, tbytes) ||
        harness_dev_alloc_copy(&dseg, stream, total)) {
        printf("FAIL %s: device allocation\n", s->name);
        return 1;
    }
    /* create_segments: a send convertor's set_position snaps each end */
    opal_convertor_prepare_for_send(&c, &dt, s->count, dsend);
    if (c.fAdvance != opal_rocm_pack) {
        printf("FAIL %s: pack not offloaded\n", s->name);
        return 1;
    }
    while (pos < total) {
        size_t end = pos + s->seg;
        opal_convertor_set_position(&c, &end);
        if (end <= pos) {
            printf("FAIL %s: set_position made no progress at %zu\n", s->name, pos);
            return 1;
        }
        segs[nseg][0] = pos;
        segs[nseg][1] = end - pos;
        ++nseg;
        pos = end;
    }
    /* shuffle_segments (position.c:96-107) */
    for (size_t i = 0; i < nseg / 2; i += 2) {
        size_t t0 = segs[i][0], t1 = segs[i][1];
        segs[i][0] = segs[nseg - i - 1][0];
        segs[i][1] = segs[nseg - i - 1][1];
        segs[nseg - i - 1][0] = t0;
        segs[nseg - i - 1][1] = t1;
    }
    /* pack_segments: fresh convertor, set_position + pack per segment */
    opal_convertor_prepare_for_send(&c, &dt, s->count, dsend);
    for (size_t i = 0; i < nseg && !fails; ++i) {
        size_t p = segs[i][0], max = segs[i][1];
        struct iovec iov = {(char *) dseg + segs[i][0], segs[i][1]};
        uint32_t n = 1;
        opal_convertor_set_position(&c, &p);
        if (p != segs[i][0] || opal_convertor_pack(&c, &iov, &n, &max) < 0 || max != segs[i][1]) {
            printf("FAIL %s: pack segment %zu (%zu at %zu): position %zu, max %zu\n", s->name, i,
                   segs[i][1], segs[i][0], p, max);
            ++fails;
        }
    }
    if (!fails && (harness_dev_copy_back(pk, dseg, total) || memcmp(pk, stream, total))) {
        size_t bad = 0;
        while (bad < total && pk[bad] == stream[bad]) ++bad;
        printf("FAIL %s: packed segments differ from the oracle's stream at byte %zu\n", s->name, bad);
        ++fails;
    }
    /* unpack_segments: fresh receive convertor, same order */
    opal_convertor_prepare_for_recv(&c, &dt, s->count, drecv);
    for (size_t i = 0; i < nseg && !fails; ++i) {
        size_t p = segs[i][0], max = segs[i][1];
        struct iovec iov = {(char *) dseg + segs[i][0], segs[i][1]};
        uint32_t n = 1;
        opal_convertor_set_position(&c, &p);
        if (p != segs[i][0] || opal_convertor_unpack(&c, &iov, &n, &max) < 0 || max != segs[i][1]) {
            printf("FAIL %s: unpack segment %zu\n", s->name, i);
            ++fails;
        }
    }
    if (!fails && (harness_dev_copy_back(got, drecv, tbytes) || memcmp(got, exp, tbytes))) {
        size_t bad = 0;
        while (bad < tbytes && got[bad] == exp[bad]) ++bad;
        printf("FAIL %s: received typed buffer differs at byte %zu\n", s->name, bad);
        ++fails;
    }
    if (!fails) printf("ok %s (%zu segments)\n", s->name, nseg);
    harness_dev_free(dsend);
    harness_dev_free(drecv);
    harness_dev_free(dseg);
    free(segs); free(typed); free(bg); free(stream); free(got); free(exp); free(pk);
    return fails;
}

/* HARNESS_BENCH=1: the per-fragment cost of the seam measured from C, the
 * way a PML drives it — 64 KiB fragments (ob1's default max send size)
 * over a 256 MiB packed stream of MPI_Type_vector(blocklen 8 doubles,
 * stride 16): one fAdvance per fragment, synchronous (device fragments),
 * deferred (opal_rocm_set_copy_function_async + one record_event), and host
 * fragments (pageable memory, btl/sm-style); against one fAdvance over the
 * whole fragment train (iov_batch).  One JSON line per (mode, direction). */
#include <time.h>
static double now_s(void)
{
    struct timespec t;
    clock_gettime(CLOCK_MONOTONIC, &t);
    return (double) t.tv_sec + 1e-9 * (double) t.tv_nsec;
}

static int bench(void)
{
    const size_t frag = 64 << 10, total = (size_t) 256 << 20, nfrag = total / frag;
    const size_t nblk = total / 64, tbytes = nblk * 128;
    dt_elem_desc_t desc[2];
    opal_datatype_t dt;
    memset(desc, 0, sizeof(desc));
    desc[0].elem.common.type = OPAL_DATATYPE_FLOAT8;
    desc[0].elem.common.flags = OPAL_DATATYPE_FLAG_DATA;
    desc[0].elem.count = (uint32_t) nblk;
    desc[0].elem.blocklen = 8;
    desc[0].elem.extent = 128;
    desc[1].end_loop.common.type = OPAL_DATATYPE_END_LOOP;
    desc[1].end_loop.items = 1;
    desc[1].end_loop.size = total;
    memset(&dt, 0, sizeof(dt));
    dt.size = total;
    dt.ub = dt.true_ub = (ptrdiff_t) tbytes;
    dt.opt_desc.used = dt.opt_desc.length = 2;
    dt.opt_desc.desc = desc;
    void *dtyped = NULL, *dpack = NULL;
    char *zero = calloc(tbytes, 1), *hpack = malloc(total);
    struct iovec *all = malloc(nfrag * sizeof(*all));
    if (harness_dev_alloc_copy(&dtyped, zero, tbytes) || harness_dev_alloc_copy(&dpack, zero, total)) {
        printf("FAIL bench alloc\n");
        return 1;
    }
    memset(hpack, 1, total);
    const char *modes[] = {"per_fragment_sync", "per_fragment_deferred", "host_fragments", "iov_batch"};
    for (int m = 0; m < 4; ++m)
        for (int dir = 0; dir < 2; ++dir) {
            double best = 1e30;
            for (int rep = 0; rep < 3; ++rep) {
                opal_convertor_t c;
                char *base = m == 2 ? hpack : (char *) dpack;
                void *ev = NULL;
                if (dir == 0) opal_convertor_prepare_for_send(&c, &dt, 1, dtyped);
                else opal_convertor_prepare_for_recv(&c, &dt, 1, dtyped);
                if (m == 1) opal_rocm_set_copy_function_async(&c, NULL);
                ompi_amd_stream_synchronize(NULL);
                const double t0 = now_s();
                if (m == 3) {
                    for (size_t k = 0; k < nfrag; ++k) {
                        all[k].iov_base = base + k * frag;
                        all[k].iov_len = frag;
                    }
                    uint32_t n = (uint32_t) nfrag;
                    size_t max = total;
                    if ((dir ? opal_convertor_unpack(&c, all, &n, &max) : opal_convertor_pack(&c, all, &n, &max)) != 1)
                        printf("FAIL bench iov_batch\n");
                } else {
                    for (size_t k = 0; k < nfrag; ++k) {
                        struct iovec v = {base + k * frag, frag};
                        uint32_t n = 1;
                        size_t max = frag;
                        if ((dir ? opal_convertor_unpack(&c, &v, &n, &max) : opal_convertor_pack(&c, &v, &n, &max)) < 0) {
                            printf("FAIL bench fragment %zu\n", k);
                            break;
                        }
                    }
                    if (m == 1) {
                        opal_rocm_record_event(&c, &ev);
                        ompi_amd_event_synchronize(ev);
                        ompi_amd_event_destroy(ev);
                    }
                }
                ompi_amd_stream_synchronize(NULL);
                const double t = now_s() - t0;
                if (t < best) best = t;
                opal_rocm_convertor_release(&c);
            }
            /* algorithmic bytes: the packed stream read / written once and
             * its typed span (2x, blocks 64 of every 128 B) the other way */
            printf("{\"bench\": \"ddt_fragments\", \"mode\": \"%s\", \"dir\": \"%s\", "
                   "\"fragments\": %zu, \"fragment_bytes\": %zu, \"seconds\": %.6f, "
                   "\"us_per_fragment\": %.3f, \"packed_GBps\": %.1f, \"algorithmic_GBps\": %.1f, "
                   "\"cuda_support_build\": %d}\n",
                   modes[m], dir ? "unpack" : "pack", nfrag, frag, best, 1e6 * best / (double) nfrag,
                   (double) total / best / 1e9, 2.0 * (double) total / best / 1e9, OPAL_CUDA_SUPPORT);
        }
    harness_dev_free(dtyped);
    harness_dev_free(dpack);
    free(zero);
    free(hpack);
    free(all);
    return 0;
}

int main(void)
{
    static const struct { int type; size_t size; } sizes[] = {
        {OPAL_DATATYPE_INT1, 1}, {OPAL_DATATYPE_INT2, 2}, {OPAL_DATATYPE_INT4, 4},
        {OPAL_DATATYPE_INT8, 8}, {OPAL_DATATYPE_UINT1, 1}, {OPAL_DATATYPE_FLOAT4, 4},
        {OPAL_DATATYPE_FLOAT8, 8}, {OPAL_DATATYPE_FLOAT16, 16}};
    for (size_t i = 0; i < sizeof(sizes) / sizeof(sizes[0]); ++i) {
        basic[sizes[i].type].size = sizes[i].size;
        opal_datatype_basicDatatypes[sizes[i].type] = &basic[sizes[i].type];
    }
    const int gpu = getenv("HARNESS_GPU") && atoi(getenv("HARNESS_GPU"));
#if OPAL_CUDA_SUPPORT
    opal_cuda_add_initialization_function(mca_common_rocm_fill_table);
#else
    gpu_enabled = gpu;  /* nothing to register: the seam asks the runtime itself */
#endif
    if (!gpu) {
        /* no GPU: the table must refuse, nothing may be offloaded */
        static char host_buf[64];
        opal_datatype_t dt;
        memset(&dt, 0, sizeof(dt));
        dt.size = 8;
        dt.ub = 16;
        opal_convertor_t c;
        opal_convertor_prepare_for_send(&c, &dt, 2, host_buf);
        if (gpu_enabled || (c.flags & CONVERTOR_CUDA) || c.fAdvance) {
            printf("FAIL: offload selected without a GPU\n");
            return 1;
        }
        printf("ok cpu (OPAL_CUDA_SUPPORT %d)\n", OPAL_CUDA_SUPPORT);
        return 0;
    }
#if OPAL_CUDA_SUPPORT
    if (!gpu_enabled) {
        printf("FAIL: mca_common_rocm_fill_table refused on a GPU host\n");
        return 1;
    }
#endif
    if (getenv("HARNESS_BENCH") && atoi(getenv("HARNESS_BENCH"))) return bench();
    {   /* a host buffer is never offloaded (either build) */
        static char host_buf[64];
        opal_datatype_t dt;
        opal_convertor_t c;
        memset(&dt, 0, sizeof(dt));
        dt.size = 8;
        dt.ub = 16;
        opal_convertor_prepare_for_send(&c, &dt, 2, host_buf);
        if (c.fAdvance) {
            printf("FAIL: a host buffer was offloaded\n");
            return 1;
        }
    }
    {   /* a description the device program cannot hold (6000 flattened
         * runs > FLAT_MAX_ELEMS) on device memory: a CUDA-support build keeps
         * the reference's walker (its cbmemcpy copies device runs); a
         * ROCm-only build must fail the conversion without the CPU touching
         * the device buffer */
        opal_datatype_t dt;
        dt_elem_desc_t desc[4];
        opal_convertor_t c;
        void *dbuf = NULL;
        char *zero = calloc(3000 * 64, 1), host[256];
        struct iovec iov = {host, sizeof(host)};
        uint32_t n = 1;
        size_t max = sizeof(host);
        memset(&dt, 0, sizeof(dt));
        memset(desc, 0, sizeof(desc));
        desc[0].loop.common.type = OPAL_DATATYPE_LOOP;
        desc[0].loop.items = 3;
        desc[0].loop.loops = 3000;
        desc[0].loop.extent = 64;
        for (int k = 0; k < 2; ++k) {
            desc[1 + k].elem.common.type = OPAL_DATATYPE_FLOAT8;
            desc[1 + k].elem.common.flags = OPAL_DATATYPE_FLAG_DATA;
            desc[1 + k].elem.count = 1;
            desc[1 + k].elem.blocklen = 1;
            desc[1 + k].elem.extent = 8;
            desc[1 + k].elem.disp = k ? 24 : 0;
        }
        desc[3].end_loop.common.type = OPAL_DATATYPE_END_LOOP;
        desc[3].end_loop.items = 3;
        desc[3].end_loop.size = 16;
        dt.size = 3000 * 16;
        dt.ub = 3000 * 64;
        dt.true_ub = 2999 * 64 + 32;
        dt.opt_desc.desc = desc;
        dt.opt_desc.used = 4;
        dt.desc = dt.opt_desc;
        if (harness_dev_alloc_copy(&dbuf, zero, 3000 * 64) != 0) {
            printf("FAIL: device alloc\n");
            return 1;
        }
        memset(host, 0x5A, sizeof(host));
        opal_convertor_prepare_for_send(&c, &dt, 1, dbuf);
#if OPAL_CUDA_SUPPORT
        (void) iov;
        (void) n;
        (void) max;
        if (opal_rocm_convertor_owns(&c)) {
            printf("FAIL: an unflattenable description was offloaded\n");
            return 1;
        }
#else
        if (c.fAdvance != opal_rocm_refuse || opal_convertor_pack(&c, &iov, &n, &max) != -1 ||
            max != 0 || (unsigned char) host[0] != 0x5A) {
            printf("FAIL: an unflattenable device description was not refused\n");
            return 1;
        }
#endif
        printf("ok unflattenable device description (OPAL_CUDA_SUPPORT %d)\n", OPAL_CUDA_SUPPORT);
        harness_dev_free(dbuf);
        free(zero);
    }
    int fails = 0, types = 0;
    spec_t s;
    int r;
    while ((r = read_spec(stdin, &s)) == 1) {
        fails += (s.kind == 'U' ? test_unpack_ooo(&s) : s.kind == 'P' ? test_position(&s) : test_type(&s)) ? 1 : 0;
        ++types;
        free(s.blocks);
        free(s.desc);
        free(s.init);
        free(s.packed);
        free(s.expect);
    }
    if (r < 0) {
        printf("FAIL: bad spec after %d types\n", types);
        return 1;
    }
    printf("programs cached %d (OPAL_CUDA_SUPPORT %d)\n", opal_rocm_program_cache_size(), OPAL_CUDA_SUPPORT);
    opal_rocm_program_cache_clear();
    if (fails) printf("FAILED %d of %d\n", fails, types);
    else printf("all %d ok\n", types);
    return fails ? 1 : 0;
}
