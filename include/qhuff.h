/*
 * qhuff.h -- C-ABI of the MI355X-native QPACK Huffman string-literal codec.
 *
 * Drop-in boundary for the string-literal step of ls-qpack (v2.6.5).  The
 * reference codes one string per synchronous call:
 *
 *   lsqpack_enc_enc_str()      lsqpack.c:839-876   (test/lsqpack-test.h:17-19)
 *   qenc_enc_str_size()        lsqpack.c:5198-5210 (static; ratio guard 1946)
 *   qenc_huffman_enc()         lsqpack.c:5085-5195 (static)
 *   lsqpack_huff_decode()      lsqpack.c:3520-3535 (LSQPACK_DEVEL_MODE export)
 *   lsqpack_huff_decode_full() lsqpack.c:3443-3517 (exported)
 *
 * This library codes a BATCH of independent strings per call on one GPU.
 * Every entry point is plain C: pointers, sizes, status codes.  No HIP or
 * torch types cross this header; `stream` is an opaque hipStream_t (NULL =
 * the device's default stream).
 *
 * Batch layout (device memory unless a function says host):
 *   in      strings packed back to back.
 *   in_off  n + 1 uint32 exclusive offsets: string i is
 *           in[in_off[i] .. in_off[i+1]).  in_off[0] need not be 0.
 *   out     packed outputs; out_off (n + 1 entries) is written by the call:
 *           output i is out[out_off[i] .. out_off[i+1]), out_off[0] = 0.
 *
 * Results are bit-exact with the reference functions named on each call.
 * Failure is loud: a call returns a negative QHUFF_E* code, and the library
 * has no CPU fallback -- without a usable gfx950 device qhuff_open fails.
 */
#ifndef QHUFF_H
#define QHUFF_H 1

#include <stddef.h>
#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

/* ABI versions:
 *   1  batch encode / decode, host path, per-string mirrors.  (An early
 *      header of this version declared qhuff_huff_decode with 7 arguments,
 *      state and final included; the symbol takes 5 -- a caller built
 *      against that header links but its state / final are ignored: use
 *      qhuff_huff_decode_ex and check qhuff_abi_version() >= 2.)
 *   2  qhuff_huff_decode_ex (the reference's full argument list) beside the
 *      5-argument qhuff_huff_decode, which is unchanged
 *   3  the low-latency service (qhuff_svc_*) and, in qhuff_lsqpack.h,
 *      qhuff_lsqpack_set_context
 *   4  launch timing (qhuff_timing_enable / qhuff_timing_read)
 *   5  qhuff_kernel_variant (which kernel variant the last launch ran);
 *      qhuff_timing_enable(ctx, k > 1) samples every k-th launch
 *   6  QHUFF_MAX_STRLEN: qhuff_scan_field_section rejects (QHUFF_EPROTO) a
 *      literal whose declared length exceeds it; qhuff_decode_literals_ex
 *      rejects a literal whose decoded length does; qhuff_batch_hint /
 *      qhuff_batch_needs_full (the kernel variant from the batch)
 *   7  qhuff_dec_int (the pre-parse's integer decoder); qhuff_decode_
 *      literals_ex applies max_len to a field line's name + value;
 *      qhuff_encode_batch_host_multi / qhuff_decode_batch_host_multi and
 *      qhuff_*_batch_multi (one batch over several contexts / GPUs); an
 *      unhinted launch runs the full kernel (decode's launch history is
 *      gone); qhuff_host_register / qhuff_host_unregister (direct DMA for
 *      the host-memory calls) */
#define QHUFF_ABI_VERSION 7

/* QHUFF_ABI_VERSION of the loaded library (compare with the header's) */
int qhuff_abi_version(void);

/* return codes */
#define QHUFF_OK          0
#define QHUFF_EINVAL    (-22)   /* bad argument (NULL pointer, bad mode)   */
#define QHUFF_ENOMEM    (-12)   /* device allocation failed                */
#define QHUFF_ENODEV    (-19)   /* no usable device                        */
#define QHUFF_ERANGE    (-34)   /* batch too large for 32-bit offsets      */
#define QHUFF_EDEVICE   (-5)    /* a HIP call failed (see qhuff_last_error) */

/* encode modes (qhuff_encode_batch `mode`) */
#define QHUFF_ENC_PAYLOAD   0   /* qenc_huffman_enc output only (forced
                                   Huffman, no framing), lsqpack.c:5085   */
#define QHUFF_ENC_LITERAL3  3   /* lsqpack_enc_enc_str(3, ...) framing     */
#define QHUFF_ENC_LITERAL5  5   /* lsqpack_enc_enc_str(5, ...)             */
#define QHUFF_ENC_LITERAL7  7   /* lsqpack_enc_enc_str(7, ...)             */

/* per-string decode status (qhuff_decode_batch `status`) */
#define QHUFF_DEC_OK     0      /* HUFF_DEC_OK, lsqpack.c:3424             */
#define QHUFF_DEC_ERROR  1      /* HUFF_DEC_ERROR, lsqpack.c:3427: EOS in
                                   the data, padding > 7 bits, or padding
                                   that is not the EOS prefix              */

typedef struct qhuff_ctx qhuff_ctx;

/* Open a codec context on HIP device `device` (one context per host thread
 * per GPU).  Uploads the static Huffman tables once.  A context is not
 * thread-safe; its launches may use any streams (a launch on another stream
 * than the context's previous one is ordered after it).  Several contexts
 * may run on one GPU at once (tiles are claimed in order, so a grid need not
 * be co-resident).  Returns QHUFF_OK or QHUFF_E*. */
int qhuff_open(int device, qhuff_ctx **ctx_out);
void qhuff_close(qhuff_ctx *ctx);

/* Worst-case output bytes for an encode batch of n strings totalling
 * in_bytes (30-bit longest code, + framing for LITERAL modes). */
uint64_t qhuff_encode_bound(uint64_t in_bytes, uint32_t n, unsigned mode);

/* Worst-case output bytes for a decode batch (5-bit shortest code,
 * lsqpack.c:5072): floor(8 * in_bytes / 5). */
uint64_t qhuff_decode_bound(uint64_t in_bytes, uint32_t n);

/* Encode n strings (device pointers).
 *   mode PAYLOAD: output i = qenc_huffman_enc(string i) (lsqpack.c:5085),
 *                 exactly qenc_enc_str_size(string i) bytes (lsqpack.c:5198).
 *   mode LITERAL3/5/7: output i = the bytes lsqpack_enc_enc_str(mode, dst,
 *                 bound, string i) writes with dst[0] = 0 beforehand
 *                 (lsqpack.c:839): H bit + prefixed length + Huffman, or
 *                 H=0 + length + raw copy when Huffman is not shorter.
 *                 Bits of byte 0 above the H bit are 0; the caller ORs its
 *                 instruction bits in (as the reference's callers do).
 * `out` must hold qhuff_encode_bound(...) bytes.  Asynchronous on `stream`. */
int qhuff_encode_batch(qhuff_ctx *ctx, const uint8_t *in,
                       const uint32_t *in_off, uint32_t n, unsigned mode,
                       uint8_t *out, uint32_t *out_off, void *stream);

/* Decode n complete Huffman strings (device pointers), with the semantics of
 * lsqpack_huff_decode(src, len, dst, dst_len, &{resume 0}, final = 1)
 * (lsqpack.c:3524-3529 -> huff_decode_fast, 5243) given a dst_len that
 * cannot run out.  status[i] = QHUFF_DEC_OK or QHUFF_DEC_ERROR; an ERROR
 * string contributes 0 output bytes.  `out` must hold
 * qhuff_decode_bound(...) bytes.  Asynchronous on `stream`. */
int qhuff_decode_batch(qhuff_ctx *ctx, const uint8_t *in,
                       const uint32_t *in_off, uint32_t n, uint8_t *out,
                       uint32_t *out_off, uint8_t *status, void *stream);

/* Host-memory variants (PCIe-inclusive path: host -> pinned staging ->
 * device -> kernel -> device -> pinned -> host).  Synchronous.  in_off and
 * the returned out_off are host arrays of n + 1 entries; out must hold the
 * corresponding bound; out_off[n] is the output total. */
int qhuff_encode_batch_host(qhuff_ctx *ctx, const uint8_t *in,
                            const uint32_t *in_off, uint32_t n, unsigned mode,
                            uint8_t *out, uint32_t *out_off);
int qhuff_decode_batch_host(qhuff_ctx *ctx, const uint8_t *in,
                            const uint32_t *in_off, uint32_t n, uint8_t *out,
                            uint32_t *out_off, uint8_t *status);

/* (ABI 7) Register caller buffers for direct DMA by the host-memory calls
 * (hipHostRegister, portable to every device; process-wide).  When a host
 * call's input bytes and offsets each lie within one registered range they
 * are transferred to the device directly, without the pinned staging copy;
 * when its output buffer (the bound), offsets and statuses do, the results
 * are transferred straight into them (batches past one 4 MB staging chunk).  Register long-lived buffers once (it pins
 * their pages: milliseconds for tens of MB); the results are the same either
 * way.  qhuff_host_register: QHUFF_OK, QHUFF_EINVAL (null, 0 bytes, or ptr
 * already registered), QHUFF_ENOMEM / QHUFF_EDEVICE (the reason in
 * qhuff_last_error(NULL)).  qhuff_host_unregister: ptr as registered; no call
 * may be using it. */
int qhuff_host_register(void *ptr, size_t bytes);
int qhuff_host_unregister(void *ptr);

/* ---- low-latency service ----------------------------------------------
 * The reference codes one literal per call, a few dozen per header block
 * (lsqpack.c:3718, 3795, 4714, 4824, 4908 decode; 1983-2119 encode).  A
 * batch call pays a kernel launch, copies and a stream synchronisation; the
 * service instead keeps a kernel resident on the context's GPU (its own
 * stream; one workgroup = one CU per 12 request slots) that polls request
 * slots in pinned host memory: a call writes its strings into a free slot,
 * the kernel codes them and writes the result back into the slot.
 *
 * qhuff_svc_open: attach a service to ctx (one per context) with at least
 * `slots` request slots (0: 12; at most a quarter of the CUs' worth); its
 * kernel leaves after idle_us microseconds without a request (0: 20000) and
 * the next call starts it again.  Once attached, the context's host-path
 * calls (qhuff_*_batch_host and the per-string entry points below) that fit
 * a slot go through the service too.
 *
 * qhuff_svc_encode / qhuff_svc_decode: the arguments, outputs and return
 * codes of qhuff_encode_batch_host / qhuff_decode_batch_host; callable from
 * any number of threads at once (each call takes a free slot, waiting if
 * none is free).  A call of more than QHUFF_SVC_MAX_STRINGS strings or
 * QHUFF_SVC_MAX_BYTES input bytes runs the context's host path instead (one
 * such call at a time).  Offsets must not decrease (QHUFF_EINVAL).
 *
 * qhuff_svc_close: stop the kernel and free the service (no call may be in
 * flight); qhuff_close closes an attached service.  qhuff_svc_stats: calls
 * served by the kernel, kernel launches, calls sent to the host path. */
#define QHUFF_SVC_MAX_STRINGS 1024
#define QHUFF_SVC_MAX_BYTES   65536

typedef struct qhuff_svc qhuff_svc;

int qhuff_svc_open(qhuff_ctx *ctx, unsigned slots, unsigned idle_us,
                   qhuff_svc **svc_out);
void qhuff_svc_close(qhuff_svc *svc);
int qhuff_svc_encode(qhuff_svc *svc, const uint8_t *in, const uint32_t *in_off,
                     uint32_t n, unsigned mode, uint8_t *out,
                     uint32_t *out_off);
int qhuff_svc_decode(qhuff_svc *svc, const uint8_t *in, const uint32_t *in_off,
                     uint32_t n, uint8_t *out, uint32_t *out_off,
                     uint8_t *status);
int qhuff_svc_stats(qhuff_svc *svc, uint64_t *served, uint64_t *launches,
                    uint64_t *fallbacks);

/* ---- per-string mirrors of the reference entry points -----------------
 * Same argument meaning, return values and error behaviour as the reference
 * functions; each call runs a one-string batch on the context's GPU (no CPU
 * fallback).  Host pointers.  Synchronous. */

/* lsqpack_enc_enc_str (lsqpack.c:839): returns bytes written or -1 when
 * dst_len is too small.  Bits of dst[0] above prefix_bits+1 are kept. */
int qhuff_enc_enc_str(qhuff_ctx *ctx, unsigned prefix_bits,
                      unsigned char *dst, size_t dst_len,
                      const unsigned char *str, unsigned str_len);

/* qenc_enc_str_size (lsqpack.c:5198): Huffman size in bytes. */
unsigned qhuff_enc_str_size(qhuff_ctx *ctx, const unsigned char *str,
                            unsigned str_len);

/* struct huff_decode_retval (lsqpack.c:3420-3431) */
enum qhuff_huff_dec_status
{
    QHUFF_HUFF_DEC_OK,
    QHUFF_HUFF_DEC_END_SRC,
    QHUFF_HUFF_DEC_END_DST,
    QHUFF_HUFF_DEC_ERROR
};

struct qhuff_decode_retval
{
    enum qhuff_huff_dec_status  status;
    unsigned                    n_dst;
    unsigned                    n_src;
};

/* struct lsqpack_decode_status / lsqpack_huff_decode_state (lsqpack.h:
 * 747-757), same layout */
struct qhuff_decode_status
{
    uint8_t state;
    uint8_t eos;
};

struct qhuff_huff_decode_state
{
    int                         resume;
    struct qhuff_decode_status  status;
};

/* lsqpack_huff_decode(src, src_len, dst, dst_len, state, final)
 * (lsqpack.c:3524) on context ctx: complete strings (resume == 0 && final)
 * on the GPU -- OK, ERROR with n_dst = n_src = 0, or END_DST with the
 * reference's byte-boundary back-off (lsqpack.c:5438-5450) when dst_len is
 * too small; streaming input through the decoder registered with
 * qhuff_lsqpack_set_decode_full (qhuff_lsqpack.h, which documents the exact
 * semantics). */
struct qhuff_decode_retval
qhuff_huff_decode_ex(qhuff_ctx *ctx, const unsigned char *src, int src_len,
                     unsigned char *dst, int dst_len,
                     struct qhuff_huff_decode_state *state, int final);

/* (ABI 1) a complete string: qhuff_huff_decode_ex with a zeroed state and
 * final = 1 -- OK, ERROR with n_dst = n_src = 0, or END_DST with the
 * reference's partial progress when dst_len is too small */
struct qhuff_decode_retval
qhuff_huff_decode(qhuff_ctx *ctx, const unsigned char *src, int src_len,
                  unsigned char *dst, int dst_len);

/* ---- literal-span pre-parse + batched literal decode (SURVEY.md 8(f)
 * rank 3).  A host pass walks only the instruction framing of QPACK wire
 * data -- field sections (RFC 9204 4.5; the reference's parse_header_prefix /
 * parse_header_data, lsqpack.c:3955-4046, 3567-3915) and encoder-stream
 * instructions (RFC 9204 4.3; lsqpack_dec_enc_in, lsqpack.c:4574-4960) --
 * with the reference's integer rules (lsqpack_dec_int / _int24,
 * lsqpack.c:2372-2460), and records every string literal.  Indices are not
 * resolved: the dynamic table stays with the reference.  The literals of
 * any number of blocks are then decoded in one GPU launch. */
#define QHUFF_EPROTO    (-71)   /* malformed instruction (bad integer)     */
#define QHUFF_ETRUNC    (-61)   /* input ends inside an instruction        */

#define QHUFF_LIT_NAME   1
#define QHUFF_LIT_VALUE  2

/* LSXPACK_MAX_STRLEN (lsxpack_header.h:12-13): the longest name or value a
 * field section may carry.  The reference rejects a field-section literal
 * whose declared length exceeds it right after the length integer
 * (lsqpack.c:3682-3685 values, 3769-3772 names) and a decoded one that
 * outgrows it (header_out_grow_buf, lsqpack.c:3350-3351). */
#define QHUFF_MAX_STRLEN 65535u

struct qhuff_literal
{
    uint32_t pos;               /* payload offset: pos_base + offset in buf */
    uint32_t len;               /* payload bytes                            */
    uint8_t  huffman;           /* H bit                                    */
    uint8_t  prefix_bits;       /* 3, 5 or 7: its length prefix             */
    uint8_t  kind;              /* QHUFF_LIT_NAME / QHUFF_LIT_VALUE         */
    uint8_t  hdr_len;           /* bytes of H bit + prefixed length: the
                                   literal's wire bytes are
                                   [pos - hdr_len, pos + len)                */
    uint32_t instr;             /* pos_base + offset of its instruction     */
};

/* One complete encoded field section (prefix + field lines).  Writes up to
 * max_lits literals in wire order and the count to *n_lits.  QHUFF_OK,
 * QHUFF_ETRUNC (ends inside a line), QHUFF_EPROTO (an integer the reference
 * rejects, or (ABI 6) a literal length above QHUFF_MAX_STRLEN, reported as
 * soon as the length is decoded, whether or not its bytes follow),
 * QHUFF_ERANGE (*n_lits is the count needed). */
int qhuff_scan_field_section(const uint8_t *buf, size_t len, uint32_t pos_base,
                             struct qhuff_literal *lits, uint32_t max_lits,
                             uint32_t *n_lits);

/* Encoder-stream bytes (may end inside an instruction: *consumed is the
 * length of the complete instructions, whose literals are reported; the
 * caller keeps the rest for the next chunk, as the reference resumes). */
int qhuff_scan_encoder_stream(const uint8_t *buf, size_t len,
                              uint32_t pos_base, struct qhuff_literal *lits,
                              uint32_t max_lits, uint32_t *n_lits,
                              size_t *consumed);

/* (ABI 7) The scanners' prefixed-integer decoder (RFC 7541 5.1) with the
 * reference's rules: lsqpack_dec_int (lsqpack.c:2372-2437) given the whole
 * integer in one buffer.  prefix_bits 1..8; the bits of buf[0] above the
 * prefix are ignored.  QHUFF_OK with *value and *consumed (the integer's
 * bytes), QHUFF_ETRUNC when buf ends inside the integer (the reference's -1),
 * QHUFF_EPROTO when the value does not fit 64 bits or the integer runs past
 * 10 continuation bytes (its -2). */
int qhuff_dec_int(const uint8_t *buf, size_t len, unsigned prefix_bits,
                  uint64_t *value, size_t *consumed);

/* Output bytes qhuff_decode_literals_host may write for these literals. */
uint64_t qhuff_literals_bound(const struct qhuff_literal *lits, uint32_t n);

/* Decode n literals whose payloads lie in host buffer `buf` (lits[i].pos is
 * relative to buf): Huffman ones (H = 1) on the GPU in one batch, with the
 * lsqpack_huff_decode semantics of qhuff_decode_batch; raw ones copied.
 * Host out_off[n + 1], status[n] (QHUFF_DEC_OK / QHUFF_DEC_ERROR, an ERROR
 * literal contributes 0 bytes).  `out` holds qhuff_literals_bound bytes.
 * Synchronous. */
int qhuff_decode_literals_host(qhuff_ctx *ctx, const uint8_t *buf,
                               const struct qhuff_literal *lits, uint32_t n,
                               uint8_t *out, uint32_t *out_off,
                               uint8_t *status);

/* (ABI 6) qhuff_decode_literals_host with a length limit: a literal whose
 * decoded (Huffman) or raw length exceeds max_len gets QHUFF_DEC_ERROR and
 * 0 bytes.  Field-section literals take max_len = QHUFF_MAX_STRLEN (the
 * reference's header_out_grow_buf rule, lsqpack.c:3350-3351: a string
 * never outgrows LSXPACK_MAX_STRLEN); 0 = no limit (encoder-stream literals,
 * whose bound is the dynamic table's capacity, lsqpack.c:4661-4667). */
int qhuff_decode_literals_ex(qhuff_ctx *ctx, const uint8_t *buf,
                             const struct qhuff_literal *lits, uint32_t n,
                             uint32_t max_len, uint8_t *out, uint32_t *out_off,
                             uint8_t *status);

/* ---- encoder-side hook ---------------------------
 * lsqpack_enc_enc_str (lsqpack.c:839-876) for a string whose Huffman
 * payload was precomputed by a QHUFF_ENC_PAYLOAD batch (huff, huff_len =
 * that batch's output i; huff_len is also qenc_enc_str_size, the figure the
 * ratio guard at lsqpack.c:1946-1957 reads).  Same bytes, return value and
 * -1 on short dst_len as the reference; bits of dst[0] above the H bit are
 * kept.  Host-only, no device call: a patched lsqpack.c calls it per literal
 * after batch-encoding every name and value of a header list up front
 * (INTEGRATION.md). */
int qhuff_frame_literal(unsigned prefix_bits, unsigned char *dst,
                        size_t dst_len, const unsigned char *str,
                        unsigned str_len, const unsigned char *huff,
                        unsigned huff_len);

/* ---- header hashing ---------------------
 * XXH32 (deps/xxhash/xxhash.c) of header names and values, as the reference
 * computes it for every header it encodes (lsqpack.c:1681-1685) or decodes
 * (lsqpack.c:3268-3269, 3308-3309), seeded with LSQPACK_XXH_SEED
 * (lsqpack.c:623) to index its static and dynamic tables. */
#define QHUFF_XXH_SEED 39378473u

/* n headers (device pointers); header i is name in[off[2i] .. off[2i+1])
 * followed by value in[off[2i+1] .. off[2i+2]) (2n + 1 offsets, the name /
 * value layout of an lsxpack_header buffer).  Writes
 *   name_hash[i]    = XXH32(name,  name_len,  seed)
 *   nameval_hash[i] = XXH32(value, value_len, name_hash[i]).
 * Asynchronous on `stream`. */
int qhuff_xxh32_headers(qhuff_ctx *ctx, const uint8_t *in,
                        const uint32_t *off, uint32_t n, uint32_t seed,
                        uint32_t *name_hash, uint32_t *nameval_hash,
                        void *stream);

/* n independent strings (device pointers, n + 1 offsets as in the codec
 * batches): hash[i] = XXH32(string i, seed).  Asynchronous on `stream`. */
int qhuff_xxh32_batch(qhuff_ctx *ctx, const uint8_t *in,
                      const uint32_t *in_off, uint32_t n, uint32_t seed,
                      uint32_t *hash, void *stream);

/* Host-memory variant of qhuff_xxh32_headers (pinned staging, H2D, kernel,
 * D2H; synchronous): off is a host array of 2n + 1 offsets into in. */
int qhuff_xxh32_headers_host(qhuff_ctx *ctx, const uint8_t *in,
                             const uint32_t *off, uint32_t n, uint32_t seed,
                             uint32_t *name_hash, uint32_t *nameval_hash);

/* Last HIP error string for this context (diagnostics); with ctx == NULL,
 * the reason of the calling thread's last failed qhuff_open. */
const char *qhuff_last_error(qhuff_ctx *ctx);

/* Synchronise the device and return (then clear) the context's sticky device
 * error word: 0 = no error; QHUFF_DEVERR_SPIN = a look-back wait gave up;
 * QHUFF_DEVERR_RANGE = an output offset passed 2^32 (outputs of that launch
 * are invalid).  Negative QHUFF_E* on HIP failure.  The asynchronous batch
 * calls also report such an error: the next qhuff_encode_batch /
 * qhuff_decode_batch on the context returns QHUFF_EDEVICE (and clears it)
 * once the launch that hit it has completed. */
#define QHUFF_DEVERR_SPIN 1
#define QHUFF_DEVERR_RANGE 2
int qhuff_device_error(qhuff_ctx *ctx);

/* Diagnostic: in a QHUFF_PROFILE build (libqhuff_prof.so) copy up to
 * max_words per-wave phase stamps of the last launch into dst and return
 * the number available; 0 in normal builds.  Synchronous. */
uint64_t qhuff_profile_read(qhuff_ctx *ctx, uint64_t *dst, uint64_t max_words);

/* Launch timing.  With timing on, every encode / decode / hash launch of
 * the context is dispatched with a pair of HIP events that carry the
 * dispatch's own start and end timestamps (hipExtLaunchKernel: the kernel's
 * device time, what rocprofv3's kernel trace reports, with no timing
 * packets queued around the launch), kept in a ring of the last
 * QHUFF_TIMING_SLOTS launches.  qhuff_timing_read waits for them and
 * returns, oldest first, the launches timed since timing was enabled or
 * last read (at most `max`, the most recent ones): kind[i] (QHUFF_KIND_*)
 * and us[i], microseconds.  qhuff_timing_enable(ctx, 0) turns it off;
 * `on` = k > 1 (ABI 5) times only every k-th launch of each kind, counted
 * from the call (a timed launch costs a few microseconds of queue time).
 * Return QHUFF_OK / the count, or QHUFF_E*. */
#define QHUFF_TIMING_SLOTS 256
#define QHUFF_KIND_ENCODE 0
#define QHUFF_KIND_DECODE 1
#define QHUFF_KIND_HASH   2
int qhuff_timing_enable(qhuff_ctx *ctx, int on);
int qhuff_timing_read(qhuff_ctx *ctx, uint32_t *kind, double *us, uint32_t max);

/* Kernel variants.  Encode and decode each have a lean kernel and a full
 * one that also carries the big-tile slots and the cooperative long-string
 * decode.  By default (QHUFF_KERNELS=auto) a launch runs the full kernel,
 * unless its batch is known to need only the lean one: the host-memory calls
 * read their offsets, a device-pointer caller may pass a hint (below);
 * QHUFF_KERNELS=lean|full pins one.  (Until ABI 6 decode chose by a history
 * of earlier launches.)  Returns 1 if the context's last launch of `kind`
 * (QHUFF_KIND_ENCODE / QHUFF_KIND_DECODE) ran the full kernel, 0 if the
 * lean one or none yet, QHUFF_EINVAL otherwise.  Diagnostic: the output
 * bytes are the same either way. */
int qhuff_kernel_variant(qhuff_ctx *ctx, int kind);

/* (ABI 6) The variant of the next launch of `kind` from what the caller
 * knows of its batch: hint 1 = the batch has
 * a string longer than 128 bytes or a 64-string tile spanning more than the
 * kernels' 3 KB stage (the full kernel), 0 = it has none (the lean one),
 * -1 = no hint.  Applies to the next launch of that kind only.  The host-
 * memory calls (qhuff_*_batch_host, qhuff_decode_literals_*) set it
 * themselves from the offsets they hold; a caller of the device-pointer
 * calls that keeps a host copy of its offsets (e.g. from
 * qhuff_scan_field_section) can compute it with qhuff_batch_needs_full. */
int qhuff_batch_hint(qhuff_ctx *ctx, int kind, int hint);

/* 1 if host offsets in_off[n + 1] describe a batch the full kernel is for
 * (the rule above), 0 if not, QHUFF_EINVAL for a null pointer.  Host only. */
int qhuff_batch_needs_full(const uint32_t *in_off, uint32_t n);

/* ---- multi-GPU sharding helpers (host arithmetic only) ----------------
 * Byte-balanced contiguous partition of a batch into g shards: writes
 * g + 1 string indices to cuts (cuts[0] = 0, cuts[g] = n) so shard k holds
 * strings [cuts[k], cuts[k+1]) with roughly equal input bytes
 * (SURVEY.md section 8(e)). */
int qhuff_shard_cuts(const uint32_t *in_off, uint32_t n, uint32_t g,
                     uint32_t *cuts);

/* (ABI 7) One batch over g contexts -- one per GPU, or several on one GPU
 * (distinct contexts; none in use by another thread during the call).  The
 * path shards trivially (a string's output depends only on its own bytes,
 * lsqpack.c:5085-5195, 5234-5466): the batch is cut by qhuff_shard_cuts
 * into g contiguous shards, shard k runs on ctxs[k] on a host thread of its
 * own (the calling thread takes shard 0), and the outputs are stitched by
 * each shard's base, the exclusive scan of the shard totals.  No
 * collective.
 *
 * Host memory: the arguments, outputs and return codes of
 * qhuff_encode_batch_host / qhuff_decode_batch_host on one context, and the
 * same bytes (out_off is global).  Each shard's uploads, kernels and
 * downloads run unsynchronised; only its copies into `out` wait for the
 * earlier shards' totals.  Synchronous. */
int qhuff_encode_batch_host_multi(qhuff_ctx *const *ctxs, uint32_t g,
                                  const uint8_t *in, const uint32_t *in_off,
                                  uint32_t n, unsigned mode, uint8_t *out,
                                  uint32_t *out_off);
int qhuff_decode_batch_host_multi(qhuff_ctx *const *ctxs, uint32_t g,
                                  const uint8_t *in, const uint32_t *in_off,
                                  uint32_t n, uint8_t *out, uint32_t *out_off,
                                  uint8_t *status);

/* Device-resident shards (shard k in ctxs[k]'s device memory, laid out as
 * for qhuff_encode_batch / qhuff_decode_batch; status unused by encode;
 * stream: an opaque hipStream_t of that device, NULL = its default stream).
 * Launches every shard, waits for them, and writes base[0 .. g]: base[k] =
 * the output bytes of shards [0, k), base[g] the total.  rebase != 0: shard
 * k's out_off (n_k + 1 entries) is also rebased by base[k] on its device, so
 * that it indexes the concatenation of the shards' outputs (the stitched
 * batch; the total must fit 32 bits, else QHUFF_ERANGE).  Synchronous. */
struct qhuff_shard
{
    const uint8_t  *in;
    const uint32_t *in_off;
    uint32_t        n;
    uint8_t        *out;
    uint32_t       *out_off;
    uint8_t        *status;
    void           *stream;
};
int qhuff_encode_batch_multi(qhuff_ctx *const *ctxs, uint32_t g,
                             const struct qhuff_shard *shards, unsigned mode,
                             uint64_t *base, int rebase);
int qhuff_decode_batch_multi(qhuff_ctx *const *ctxs, uint32_t g,
                             const struct qhuff_shard *shards, uint64_t *base,
                             int rebase);

/* Synthetic header-string batch: xorshift64
 * seeded with `seed` (0 -> 0x9E3779B97F4A7C15); len = min_len +
 * r % (max_len - min_len + 1); bytes alphabet[r % alphabet_len].  Host
 * buffers: in_off gets n + 1 entries; data must hold n * max_len bytes.
 * Returns the total bytes written. */
uint64_t qhuff_synth_batch(uint64_t seed, uint32_t n, uint32_t min_len,
                           uint32_t max_len, const uint8_t *alphabet,
                           uint32_t alphabet_len, uint8_t *data,
                           uint32_t *in_off);

#ifdef __cplusplus
}
#endif

#endif
