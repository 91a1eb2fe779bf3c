/*
 * qhuff_lsqpack.h -- the reference's string entry points with their exact
 * argument lists, served by the MI355X codec (libqhuff.so).
 *
 *   lsqpack_enc_enc_str   lsqpack.c:839-876  (test/lsqpack-test.h:17-19)
 *   lsqpack_huff_decode   lsqpack.c:3520-3535 (LSQPACK_DEVEL_MODE export;
 *                         struct huff_decode_retval lsqpack.c:3420-3431,
 *                         struct lsqpack_huff_decode_state lsqpack.h:747-757)
 *
 * A vendored lsqpack.c resolves its call sites to these with two lines after
 * the reference definitions:
 *
 *   #define lsqpack_enc_enc_str  qhuff_lsqpack_enc_enc_str   (after line 876)
 *   #define lsqpack_huff_decode  qhuff_lsqpack_huff_decode   (after line 3535)
 *
 * Each call codes one string on the calling thread's default context (opened
 * on first use on qhuff_lsqpack_set_device()'s device, else $QHUFF_DEVICE,
 * else the current HIP device), or on the context qhuff_lsqpack_set_context
 * shares.  Without a service attached a call pays a launch and two PCIe
 * copies; with one (qhuff_svc_open on a shared context) it is one request to
 * the resident kernel.  The batch calls in qhuff.h are the fast path.
 */
#ifndef QHUFF_LSQPACK_H
#define QHUFF_LSQPACK_H 1

#include "qhuff.h"

#ifdef __cplusplus
extern "C" {
#endif

/* lsqpack_enc_enc_str(prefix_bits, dst, dst_len, str, str_len): bytes
 * written (H bit + prefixed length + Huffman or raw), or -1 when dst_len is
 * too small; bits of dst[0] above the H bit are kept. */
int qhuff_lsqpack_enc_enc_str(unsigned prefix_bits, unsigned char *dst,
                              size_t dst_len, const unsigned char *str,
                              unsigned str_len);

/* lsqpack_huff_decode(src, src_len, dst, dst_len, state, final).
 *   resume == 0 && final (a complete string, the reference's
 *   huff_decode_fast, lsqpack.c:5243): decoded on the GPU.
 *     OK       decoded length, n_src = src_len
 *     ERROR    n_dst = n_src = 0 (EOS in the data, padding >= 8 bits or not
 *              the EOS prefix)
 *     END_DST  dst too small: the output prefix and input bytes up to the
 *              last byte-aligned symbol boundary before the window that did
 *              not fit, state untouched (lsqpack.c:5438-5450), so the caller
 *              grows dst and continues from n_src.  When the reference would
 *              have reached a code longer than its 16-bit window first
 *              (lsqpack.c:5452-5465), the rest goes to the registered
 *              streaming decoder, as in the reference; with none registered
 *              the same byte-boundary END_DST is returned.
 *   otherwise (resumed or non-final chunks: streaming input): the registered
 *   streaming decoder (the reference's own lsqpack_huff_decode_full,
 *   lsqpack.c:3443, always exported); with none registered: ERROR.
 *   An invalid string gets the reference's answer too: ERROR -- or END_DST
 *   (the same byte-boundary back-off) when dst runs out before the
 *   reference reaches the error, and the streaming decoder's result where
 *   a code longer than 16 bits comes first (the GPU decodes the bytes
 *   before the error, qhuff_fastwalk.h replays the reference over them).
 * (qhuff_huff_decode_ex in qhuff.h is the same on an explicit context.) */
struct qhuff_decode_retval
qhuff_lsqpack_huff_decode(const unsigned char *src, int src_len,
                          unsigned char *dst, int dst_len,
                          struct qhuff_huff_decode_state *state,
                          int final);

/* The streaming decoder for partial input (lsqpack_huff_decode_full's
 * signature; state is struct lsqpack_huff_decode_state). */
typedef struct qhuff_decode_retval (*qhuff_huff_decode_full_fn)(
    const unsigned char *src, int src_len, unsigned char *dst, int dst_len,
    struct qhuff_huff_decode_state *state, int final);
void qhuff_lsqpack_set_decode_full(qhuff_huff_decode_full_fn fn);

/* Device of the calling thread's default context (before its first call;
 * QHUFF_EINVAL after).  Returns QHUFF_OK. */
int qhuff_lsqpack_set_device(int device);

/* Serve every thread's calls from one context instead of a default context
 * per thread (NULL: back to those).  The context must have the low-latency
 * service attached (qhuff_svc_open): it makes these one-string calls
 * thread-safe and answers them without a kernel launch per call.  The
 * caller keeps ctx open while it is set.  Returns QHUFF_OK. */
int qhuff_lsqpack_set_context(qhuff_ctx *ctx);

#ifdef __cplusplus
}
#endif

#endif
