// qhuff_shim.cpp -- the reference's per-string entry points with their exact
// argument lists (include/qhuff_lsqpack.h) and the context form of
// lsqpack_huff_decode (include/qhuff.h qhuff_huff_decode_ex).
//
// A complete string is decoded on the GPU (a one-string batch).  When the
// caller's dst is too small, or the string holds a code longer than 16 bits,
// the result the reference reports is a function of where its fast decoder's
// 16-bit windows fall (huff_decode_fast, lsqpack.c:5243-5466):
// qhuff_fastwalk.h replays that control flow over the code lengths of the
// symbols the GPU decoded -- where the output stops, how far it backs off to
// a byte boundary, or from which byte the reference's nibble decoder takes
// over.  No bit is decoded on the host.  Streaming input (resume != 0 or final == 0) stays with the
// reference's own resumable decoder, registered by the integrator
// (lsqpack_huff_decode_full, lsqpack.c:3443).
#include <hip/hip_runtime.h>

#include <stdlib.h>
#include <string.h>

#include <atomic>
#include <vector>

#include "../../include/qhuff_lsqpack.h"
#include "qhuff_fastwalk.h"
#include "qhuff_tables.h"

namespace qhuff {
bool ctx_has_service(const qhuff_ctx *c);   // (qhuff_host.cpp)
int decode_keep_rejected(qhuff_ctx *c, const uint8_t *in,
                         const uint32_t *in_off, uint32_t n, uint8_t *out,
                         uint32_t *out_off, uint8_t *status);
}

namespace {

std::atomic<qhuff_huff_decode_full_fn> g_full{nullptr};
// a context shared by every thread (qhuff_lsqpack_set_context)
std::atomic<qhuff_ctx *> g_shared{nullptr};

// the calling thread's default context (closed at thread exit)
struct ThreadCtx
{
    qhuff_ctx *ctx = nullptr;
    int device = -1;
    std::vector<unsigned char> buf;          // one-string decode output
    std::vector<uint8_t> lens;               // its code lengths
    ~ThreadCtx()
    {
        if (ctx)
            qhuff_close(ctx);
    }
};
thread_local ThreadCtx t_ctx;

qhuff_ctx *
default_ctx()
{
    if (qhuff_ctx *s = g_shared.load(std::memory_order_acquire))
        return s;
    if (!t_ctx.ctx)
    {
        int dev = t_ctx.device;
        if (dev < 0)
        {
            const char *e = getenv("QHUFF_DEVICE");
            if (e)
                dev = atoi(e);
            else if (hipGetDevice(&dev) != hipSuccess)
                dev = 0;
        }
        if (qhuff_open(dev, &t_ctx.ctx) != QHUFF_OK)
            t_ctx.ctx = nullptr;
    }
    return t_ctx.ctx;
}

constexpr qhuff_decode_retval kErr = {QHUFF_HUFF_DEC_ERROR, 0, 0};


// An invalid complete string (the GPU rejected it).  The reference reports
// ERROR (n_dst = n_src = 0, lsqpack.c:5374-5425, 3482-3497) -- unless dst
// runs out before it reaches the error, when it reports END_DST like for a
// valid string (5438-5450) or its nibble decoder does (3469-3491) -- and
// where a code longer than 16 bits sends the reference to that nibble
// decoder (5452-5465), its result (ERROR with the n_dst / n_src it reached
// when the end of the input is not a valid padding, 3502-3507) is what the
// reference returns.  The GPU decodes the string again keeping the bytes
// before the error (the Keep kernel), and fast_walk_invalid replays the
// reference over their code lengths.
qhuff_decode_retval
rejected(qhuff_ctx *c, const unsigned char *src, int src_len,
         unsigned char *dst, int dst_len, struct qhuff_huff_decode_state *state,
         int final)
{
    std::vector<unsigned char> &buf = t_ctx.buf;
    const uint32_t off[2] = {0, (uint32_t) src_len};
    uint32_t oo[2] = {0, 0};
    uint8_t st = QHUFF_DEC_OK;
    if (qhuff::decode_keep_rejected(c, src, off, 1, buf.data(), oo, &st)
            != QHUFF_OK || st != QHUFF_DEC_ERROR)
        return kErr;
    const unsigned n = oo[1];                // bytes before the error
    std::vector<uint8_t> &lens = t_ctx.lens;
    lens.resize(n + 1);
    uint64_t pbits = 0;
    for (unsigned i = 0; i < n; ++i)
    {
        lens[i] = qhuff::kLen[buf[i]];
        pbits += lens[i];
    }
    // the EOS code right after them (else the padding is what is wrong)
    const bool eos = pbits + 30 <= 8ull * (uint64_t) src_len
                  && qhuff::bits_at(src, (uint32_t) src_len, (uint32_t) pbits)
                         >> 2 == 0x3fffffffu;
    if (eos)
        lens[n] = 30;
    const qhuff::FastStop fs = qhuff::fast_walk_invalid(
        lens.data(), n + (eos ? 1 : 0), src, (uint32_t) src_len,
        (uint32_t) dst_len);
    if (fs.end == qhuff::kFastDone)
        return kErr;
    if (fs.n_dst)
        memcpy(dst, buf.data(), fs.n_dst);
    if (fs.end == qhuff::kFastSlow)
    {
        const qhuff_huff_decode_full_fn full = g_full.load();
        if (full)
        {
            // the reference's nibble decoder from that byte (5452-5465)
            qhuff_decode_retval rv = full(src + fs.n_src,
                                          src_len - (int) fs.n_src,
                                          dst + fs.n_dst,
                                          dst_len - (int) fs.n_dst, state,
                                          final);
            if (rv.status == QHUFF_HUFF_DEC_OK
                    || rv.status == QHUFF_HUFF_DEC_END_DST)
            {
                rv.n_dst += fs.n_dst;
                rv.n_src += fs.n_src;
            }
            return rv;
        }
        // no streaming decoder registered: ERROR when every byte before the
        // error fits, else the byte-boundary END_DST (as for valid strings)
        if (n <= (unsigned) dst_len)
            return kErr;
    }
    return qhuff_decode_retval{QHUFF_HUFF_DEC_END_DST, fs.n_dst, fs.n_src};
}

}  // namespace

extern "C" struct qhuff_decode_retval
qhuff_huff_decode_ex(qhuff_ctx *c, const unsigned char *src, int src_len,
                     unsigned char *dst, int dst_len,
                     struct qhuff_huff_decode_state *state, int final)
{
    if (!c || !state || src_len < 0 || dst_len < 0 || (!src && src_len)
            || (!dst && dst_len))
        return kErr;
    if (state->resume != 0 || !final)
    {
        const qhuff_huff_decode_full_fn full = g_full.load();
        return full ? full(src, src_len, dst, dst_len, state, final) : kErr;
    }
    // the whole string on the GPU
    std::vector<unsigned char> &buf = t_ctx.buf;
    const size_t cap = qhuff_decode_bound((uint64_t) src_len, 1);
    if (buf.size() < cap)
        buf.resize(cap);
    const uint32_t off[2] = {0, (uint32_t) src_len};
    uint32_t oo[2] = {0, 0};
    uint8_t st = QHUFF_DEC_ERROR;
    const unsigned char dummy = 0;
    if (qhuff_decode_batch_host(c, src_len ? src : &dummy, off, 1, buf.data(),
                                oo, &st) != QHUFF_OK)
        return kErr;
    if (st != QHUFF_DEC_OK)
        return rejected(c, src, src_len, dst, dst_len, state, final);
    const unsigned n = oo[1];
    // the code lengths decide where the reference's fast decoder stops
    std::vector<uint8_t> &lens = t_ctx.lens;
    lens.resize(n);
    bool has_long = false;
    for (unsigned i = 0; i < n; ++i)
    {
        lens[i] = qhuff::kLen[buf[i]];
        has_long |= lens[i] > 16;
    }
    qhuff::FastStop fs{qhuff::kFastDone, n, (uint32_t) src_len};
    if (n > (unsigned) dst_len || has_long)
        fs = qhuff::fast_walk(lens.data(), n, (uint32_t) src_len,
                              (uint32_t) dst_len);
    const qhuff_huff_decode_full_fn full = g_full.load();
    if (fs.end == qhuff::kFastSlow && !full && n <= (unsigned) dst_len)
        fs = qhuff::FastStop{qhuff::kFastDone, n, (uint32_t) src_len};
    if (fs.n_dst)
        memcpy(dst, buf.data(), fs.n_dst);
    if (fs.end == qhuff::kFastDone)
        return qhuff_decode_retval{QHUFF_HUFF_DEC_OK, n, (unsigned) src_len};
    if (fs.end == qhuff::kFastSlow && full)
    {
        // the reference finishes with its nibble decoder from that byte
        // (lsqpack.c:5452-5465)
        qhuff_decode_retval rv = full(src + fs.n_src, src_len - (int) fs.n_src,
                                      dst + fs.n_dst, dst_len - (int) fs.n_dst,
                                      state, final);
        if (rv.status == QHUFF_HUFF_DEC_OK || rv.status == QHUFF_HUFF_DEC_END_DST)
        {
            rv.n_dst += fs.n_dst;
            rv.n_src += fs.n_src;
        }
        return rv;
    }
    // dst_ended, or a slow-path stop with no streaming decoder registered
    return qhuff_decode_retval{QHUFF_HUFF_DEC_END_DST, fs.n_dst, fs.n_src};
}

extern "C" int
qhuff_lsqpack_enc_enc_str(unsigned prefix_bits, unsigned char *dst,
                          size_t dst_len, const unsigned char *str,
                          unsigned str_len)
{
    qhuff_ctx *c = default_ctx();
    return c ? qhuff_enc_enc_str(c, prefix_bits, dst, dst_len, str, str_len)
             : -1;
}

extern "C" struct qhuff_decode_retval
qhuff_huff_decode(qhuff_ctx *c, const unsigned char *src, int src_len,
                  unsigned char *dst, int dst_len)
{
    struct qhuff_huff_decode_state st = {0, {0, 0}};
    return qhuff_huff_decode_ex(c, src, src_len, dst, dst_len, &st, 1);
}

extern "C" int
qhuff_abi_version(void)
{
    return QHUFF_ABI_VERSION;
}

extern "C" struct qhuff_decode_retval
qhuff_lsqpack_huff_decode(const unsigned char *src, int src_len,
                          unsigned char *dst, int dst_len,
                          struct qhuff_huff_decode_state *state, int final)
{
    if (state && (state->resume != 0 || !final))
    {
        // streaming input never needs the GPU context
        const qhuff_huff_decode_full_fn full = g_full.load();
        return full ? full(src, src_len, dst, dst_len, state, final) : kErr;
    }
    qhuff_ctx *c = default_ctx();
    return c ? qhuff_huff_decode_ex(c, src, src_len, dst, dst_len, state, final)
             : kErr;
}

extern "C" void
qhuff_lsqpack_set_decode_full(qhuff_huff_decode_full_fn fn)
{
    g_full.store(fn);
}

extern "C" int
qhuff_lsqpack_set_device(int device)
{
    if (t_ctx.ctx)
        return QHUFF_EINVAL;
    t_ctx.device = device;
    return QHUFF_OK;
}

extern "C" int
qhuff_lsqpack_set_context(qhuff_ctx *ctx)
{
    // a shared context is thread-safe only through its service (qhuff_host.cpp
    // svc_call): without one, concurrent calls would race on the context's
    // host-path staging buffers and streams
    if (ctx && !qhuff::ctx_has_service(ctx))
        return QHUFF_EINVAL;
    g_shared.store(ctx, std::memory_order_release);
    return QHUFF_OK;
}
