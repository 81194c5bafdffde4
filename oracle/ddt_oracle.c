/*
 * ORACLE — TEST INFRASTRUCTURE ONLY (see oracle.h).
 *
 * Restatement of the homogeneous opal_convertor pack/unpack byte stream.
 * For a committed datatype the packed stream is the concatenation, element
 * by element (element e based at e*extent), of the typemap's contiguous
 * runs in typemap order (opal_generic_simple_pack, opal_datatype_pack.c:
 * 235-370, walking opt_desc; pack_predefined_data / pack_contiguous_loop,
 * opal_datatype_pack.h:37-206).  A convertor call with max_data = B at
 * position bConverted = P produces stream bytes [P, P+B): the reference
 * resumes mid-run and mid-predefined-element (PACK_PARTIAL_BLOCKLEN,
 * opal_datatype_pack.h:37-80; ddt_test.c:479-483 packs doubles in 12-byte
 * chunks), so a window is a plain byte range of the stream.
 * Unpack is the inverse scatter (opal_datatype_unpack.c:245-428).
 */
#include "oracle.h"

#include <string.h>

static size_t walk(const orc_block_t *blk, int nb, int64_t extent, size_t count,
                   const char *src, char *dst, size_t offset, size_t bytes,
                   int unpack)
{
    size_t elem_size = 0, total, e, done = 0, pos;
    int b;
    for (b = 0; b < nb; b++) elem_size += (size_t)blk[b].len;
    total = elem_size * count;
    if (elem_size == 0 || offset >= total) return 0;
    if (bytes > total - offset) bytes = total - offset;
    e = offset / elem_size;
    pos = offset % elem_size;
    while (done < bytes) {
        size_t run_start = 0;
        for (b = 0; b < nb && done < bytes; b++) {
            size_t len = (size_t)blk[b].len;
            if (pos < run_start + len) {
                size_t skip = pos - run_start;
                size_t n = len - skip;
                char *mem = (unpack ? dst : (char *)src) + (int64_t)e * extent + blk[b].disp + (int64_t)skip;
                if (n > bytes - done) n = bytes - done;
                if (unpack) memcpy(mem, src + done, n);
                else memcpy(dst + done, mem, n);
                done += n;
                pos += n;
            }
            run_start += len;
        }
        e++;
        pos = 0;
    }
    return done;
}

size_t orc_pack(const orc_block_t *blocks, int nblocks, int64_t extent,
                size_t count, const void *src, void *dst, size_t offset,
                size_t bytes)
{
    return walk(blocks, nblocks, extent, count, src, dst, offset, bytes, 0);
}

size_t orc_unpack(const orc_block_t *blocks, int nblocks, int64_t extent,
                  size_t count, const void *src, void *dst, size_t offset,
                  size_t bytes)
{
    return walk(blocks, nblocks, extent, count, src, dst, offset, bytes, 1);
}
