/*
 * qhuff_hook.h -- the application side of the lsqpack.c seams in
 * a memo filled by ONE GPU batch per header list
 * (encoder) or per run of received blocks (decoder), and the per-string
 * lookups a patched lsqpack.c calls before its own code.  Plain C99 over
 * include/qhuff.h; exercised by tests/c/hook_test.c.
 *
 * Encoder seam (top of lsqpack_enc_enc_str, lsqpack.c:839, and of
 * qenc_enc_str_size, lsqpack.c:5198):
 *
 *   #ifdef LSQPACK_QHUFF
 *       int r = lsqpack_qhuff_enc_lookup(prefix_bits, dst, dst_len,
 *                                        str, str_len);
 *       if (r != LSQPACK_QHUFF_MISS)
 *           return r;
 *   #endif
 *
 * Decoder seam (top of lsqpack_huff_decode, lsqpack.c:3524):
 *
 *   #ifdef LSQPACK_QHUFF
 *       struct huff_decode_retval rv;
 *       if (state->resume == 0 && final
 *               && lsqpack_qhuff_dec_lookup(src, src_len, dst, dst_len,
 *                                 (struct qhuff_decode_retval *) &rv))
 *           return rv;
 *   #endif
 *
 * A lookup answers only when its answer is the reference's own; anything
 * else is a miss and the reference code runs unchanged.
 */
#ifndef QHUFF_HOOK_H
#define QHUFF_HOOK_H 1

#include <stddef.h>

#include "qhuff.h"

#define LSQPACK_QHUFF_MISS (-2)

struct qhuff_memo;

struct qhuff_memo *qhuff_memo_new(qhuff_ctx *ctx);
void qhuff_memo_free(struct qhuff_memo *m);

/* Encoder side: Huffman payloads (QHUFF_ENC_PAYLOAD) of n strings -- every
 * name and value of the header list(s) about to be encoded -- in one launch.
 * Replaces the memo's previous encoder entries.  Lookups are keyed by the
 * (pointer, length) given here and check the bytes are unchanged. */
int qhuff_memo_encode(struct qhuff_memo *m, const unsigned char *const *strs,
                      const unsigned *lens, unsigned n);

/* Decoder side: the n literals scanned from wire buffer buf
 * (qhuff_scan_field_section / qhuff_scan_encoder_stream) in one launch.
 * Replaces the memo's previous decoder entries.  Lookups are keyed by the
 * payload pointer buf + lits[i].pos; buf must stay unchanged until then. */
int qhuff_memo_decode(struct qhuff_memo *m, const unsigned char *buf,
                      const struct qhuff_literal *lits, unsigned n);

/* The memo the calling thread's seams consult (NULL: every lookup misses). */
void lsqpack_qhuff_use(struct qhuff_memo *m);

/* lsqpack_enc_enc_str's result for a memoised string (bytes written, or -1
 * when dst_len is too small; bits of dst[0] above the H bit kept), else
 * LSQPACK_QHUFF_MISS. */
int lsqpack_qhuff_enc_lookup(unsigned prefix_bits, unsigned char *dst,
                             size_t dst_len, const unsigned char *str,
                             unsigned str_len);

/* qenc_enc_str_size's result (Huffman bytes), or -1 on a miss. */
int lsqpack_qhuff_enc_str_size(const unsigned char *str, unsigned str_len);

/* The memoised Huffman payload of str: 1 and (*huff, *huff_len), or 0. */
int lsqpack_qhuff_payload(const unsigned char *str, unsigned str_len,
                          const unsigned char **huff, unsigned *huff_len);

/* lsqpack_huff_decode(src, src_len, dst, dst_len, state{0}, final=1) for a
 * memoised literal payload: 1 with *rv (HUFF_DEC_OK, the string in dst),
 * or 0 (a miss: not memoised, invalid, or dst_len not larger than the
 * decoded length, where the reference's own END_DST rules apply). */
int lsqpack_qhuff_dec_lookup(const unsigned char *src, int src_len,
                             unsigned char *dst, int dst_len,
                             struct qhuff_decode_retval *rv);

#endif
