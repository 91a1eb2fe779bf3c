// qhuff_host.cpp -- host side of the C-ABI in include/qhuff.h: context
// (tables uploaded once, look-back workspace, error word, grid sizing),
// device-pointer batch calls, the pinned host-memory path, per-string
// mirrors of the reference entry points, and host-only helpers.
#include <hip/hip_runtime.h>

#include <stdint.h>
#include <stdio.h>
#include <stdlib.h>
#include <string.h>

#include <atomic>
#include <chrono>
#include <condition_variable>
#include <functional>
#include <mutex>
#include <new>
#include <thread>
#include <vector>

#include "qhuff_kernels.h"

// ---------------------------------------------------------------------------
// host side: context, C-ABI

using namespace qhuff;

namespace qhuff {
// qhuff_frames.cpp: a VALUE literal's static-table name length, or 0
uint32_t field_ref_name_len(const uint8_t *buf, const struct qhuff_literal &l);
}

struct DevTables
{
    uint32_t win[kWinSize];              // 16-byte aligned (copied as uint4)
    uint2 enc[257];                      // {code, bits}
    uint16_t sorted[257];
    uint16_t long2[kLong2Size];
};

// Host copy workers for the PCIe-inclusive path: a staging memcpy of tens
// of MB runs at one core's copy rate, so the pinned staging copies (and the
// out_off rebasing) are split into slices run by a few persistent threads.
struct CopyPool
{
    std::vector<std::thread> th;
    std::mutex mu;
    std::condition_variable go, done;
    std::function<void(unsigned)> job;
    unsigned slices = 0;
    std::atomic<unsigned> next{0};
    unsigned finished = 0;
    unsigned active = 0;                 // workers inside a claim loop
    uint64_t gen = 0;
    bool stop = false;

    explicit CopyPool(unsigned n)
    {
        for (unsigned i = 0; i < n; ++i)
            th.emplace_back([this] { worker(); });
    }
    ~CopyPool()
    {
        {
            std::lock_guard<std::mutex> g(mu);
            stop = true;
        }
        go.notify_all();
        for (auto &t : th)
            t.join();
    }
    void worker()
    {
        uint64_t seen = 0;
        for (;;)
        {
            std::unique_lock<std::mutex> lk(mu);
            go.wait(lk, [&] { return stop || gen != seen; });
            if (stop)
                return;
            seen = gen;
            ++active;
            const unsigned ns = slices;
            lk.unlock();
            unsigned k;
            while ((k = next.fetch_add(1)) < ns)
            {
                job(k);
                std::lock_guard<std::mutex> g(mu);
                ++finished;
            }
            std::lock_guard<std::mutex> g(mu);
            --active;
            done.notify_all();
        }
    }
    // run fn(0 .. n-1) on the workers and the calling thread; returns when
    // every slice is done
    void run(unsigned n, std::function<void(unsigned)> fn)
    {
        if (n == 0)
            return;
        if (th.empty() || n == 1)
        {
            for (unsigned k = 0; k < n; ++k)
                fn(k);
            return;
        }
        {
            std::lock_guard<std::mutex> g(mu);
            job = std::move(fn);
            slices = n;
            finished = 0;
            next.store(0);
            ++gen;
        }
        go.notify_all();
        unsigned k;
        while ((k = next.fetch_add(1)) < n)
        {
            job(k);
            std::lock_guard<std::mutex> g(mu);
            ++finished;
        }
        // every slice done AND no worker still inside its claim loop: a
        // straggler's late fetch_add can then not race the next run()'s
        // reset of job / slices / next (it reads `ns`, its own copy)
        std::unique_lock<std::mutex> lk(mu);
        done.wait(lk, [&] { return finished == n && active == 0; });
    }
    // memcpy split into ~1 MB slices
    void copy(void *dst, const void *src, size_t n)
    {
        const size_t sl = 1u << 20;
        const unsigned k = (unsigned) ((n + sl - 1) / sl);
        run(k, [=](unsigned i) {
            const size_t a = (size_t) i * sl, b = a + sl < n ? a + sl : n;
            memcpy((uint8_t *) dst + a, (const uint8_t *) src + a, b - a);
        });
    }
};

constexpr unsigned kMaxChunks = 16;          // host-path pipeline depth

struct qhuff_ctx
{
    int device;
    int n_cu;
    uint32_t enc_grid, dec_grid;         // workgroups per launch
    uint32_t hash_grid;                  // resident hash workgroups
    hipStream_t own_stream;
    DevTables *tab;                      // device
    LongParams lp;
    unsigned long long *flags;           // device look-back workspace:
                                         // tile flags [cap_tiles], super
                                         // flags [cap_super], super
                                         // accumulators [2][cap_super]
    uint32_t *err;                       // device: [0] error word, [1..3]
                                         // census, then claim counters
    uint64_t cap_tiles, cap_super;
    uint8_t *big_small;                  // device: big-tile output slots
                                         // (Coord::big) of launches of at
                                         // most kSmallGrid workgroups, lazily;
                                         // larger launches use the device's
                                         // pool (slot_pool)
    bool pool_ref;                       // holds a reference on that pool
    uint32_t max_banks;                  // pool banks it may open (1..4)
    uint32_t pool_bank;                  // 1 + the pool bank its last full
                                         // launch used (0: none yet)
    // kernel variant per kind (0 encode, 1 decode; pick_full): the full
    // kernel unless the batch is known (a hint) to need only the lean one
    bool last_full[2];                   // variant of the last launch
    int hint[2];                         // the next launch's variant from
                                         // its batch, known on the host
                                         // (host_hint), or -1: full
    int kernels;                         // QHUFF_KERNELS: 0 auto, 1 lean,
                                         // 2 full
    unsigned long long *prof;            // QHUFF_PROFILE builds: stamp buffer
    size_t prof_words;
    uint32_t epoch;
    // host-path staging
    uint8_t *h_stage;                    // pinned
    size_t h_stage_cap;
    uint8_t *d_stage;
    size_t d_stage_cap;
    // host-path pipeline: copy streams, per-chunk events, copy workers
    hipStream_t h2d_stream, d2h_stream;
    hipEvent_t ev_in[kMaxChunks], ev_k[kMaxChunks], ev_out[kMaxChunks];
    bool pipe_ready;
    CopyPool *pool;
    // launch ordering: every look-back launch records ev_last on its stream;
    // a launch on another stream waits for it first (one workspace per
    // context, whichever streams the caller and the host path use)
    hipEvent_t ev_last;
    hipStream_t last_stream;
    bool have_last;
    // pinned, device-mapped mirror of the device error word: a kernel that
    // sets an error bit also writes it here, so a batch call reports an
    // error an earlier (completed) launch left without synchronising
    uint32_t *err_host;
    uint32_t *err_host_dev;
    // the low-latency service attached by qhuff_svc_open (small host-path
    // calls on this context go through it)
    qhuff_svc *svc;
    // decode launches keep a rejected string's bytes decoded before its error
    // (qhuff::decode_keep_rejected, for qhuff_shim.cpp)
    bool keep_rejected;
    // launch timing (qhuff_timing_enable): a start / stop event pair per
    // launch, a ring of the last QHUFF_TIMING_SLOTS launches
    hipEvent_t *tev;                     // [2 * QHUFF_TIMING_SLOTS], or null
    bool t_on;
    uint32_t t_every;                    // time every t_every-th launch of
    uint64_t t_seen[3];                  // each kind (launches seen)
    uint64_t t_next, t_first;            // launches timed / first unread
    uint8_t t_kind[QHUFF_TIMING_SLOTS];
    char err_msg[256];
};

// device words: [0] sticky error word (rest reserved)
constexpr size_t kErrWords = 64;

// the calling thread's last qhuff_open failure (qhuff_last_error(NULL))
static thread_local char t_open_err[160] = "no context";

static int
fail(qhuff_ctx *c, hipError_t e, const char *what)
{
    if (c)
    {
        snprintf(c->err_msg, sizeof(c->err_msg), "%s: %s", what, hipGetErrorString(e));
        snprintf(t_open_err, sizeof(t_open_err), "%s", c->err_msg);
    }
    return e == hipErrorOutOfMemory ? QHUFF_ENOMEM : QHUFF_EDEVICE;
}

#define HIPCHK(c, call)                                                      \
    do {                                                                     \
        hipError_t e_ = (call);                                              \
        if (e_ != hipSuccess)                                                \
            return fail((c), e_, #call);                                     \
    } while (0)

// ---- big-tile output slots ---------------------------------------------------
//
// A launch in auto or full-only mode may code big tiles through kBigSlots
// global slots per wave of its grid (qhuff_pipeline.h tile_loop): 48 KB a
// wave, 151 MB for the resident grid of 256 CUs.  A launch of at most
// kSmallGrid workgroups (the per-string entry points, small batches) uses a
// region of its own context, allocated at its first such launch (4.7 MB);
// larger ones use one of the device's pool banks (up to kPoolBanks, each
// allocated at its first use, all freed with the last context that used
// the pool).  So a context's own device memory stays small (tables,
// look-back flags, its staging), however many contexts a process opens.
//
// A bank belongs to the context of its last launch.  A context launches on
// its own bank without any ordering (its own launches are ordered by
// prepare_launch); a launch on a bank another context used last first
// records the bank's event on that context's last stream and waits for it.
// A context takes a bank from another only when it has none, or when no new
// bank can be had: a context whose bank was taken from it (two contexts
// alternating -- an encode stream and a decode stream) gets a bank of its
// own, so concurrent contexts are not serialised; one context after another
// (a second context opened later) reuses the first's bank.  Nothing is
// recorded while a context keeps its bank -- an event record after every
// launch cost the bench line 4 % (683-689 against 713-720 GB/s,
// profiles/r06_c) -- and no device synchronisation is needed (it would also
// wait for other libraries' streams and a resident service kernel, ADVICE
// r05; only if recording on the last launch's stream fails, e.g. the caller
// destroyed it, is the device synchronised).  A bank outgrown by a larger
// grid is retired, not freed, until the pool's last user closes.
// (QHUFF_SLOT_BANKS=1..4 caps the banks, read at qhuff_open; 1: every
// context on one bank, the round-6 first design.)
constexpr uint32_t kSmallGrid = 8;
constexpr uint64_t kWaveSlotBytes = (uint64_t) kBigSlots * kBigSlotBytes;
constexpr int kMaxDevices = 64;
constexpr uint32_t kPoolBanks = 4;

struct SlotBank
{
    uint8_t *p = nullptr;
    uint64_t waves = 0;                  // slots for this many waves
    hipEvent_t ev = nullptr;             // (recorded when it changes hands)
    const qhuff_ctx *last_ctx = nullptr; // the last launch on it: its context
    hipStream_t last_st = nullptr;       // and stream
};

struct SlotPool
{
    std::mutex mu;
    SlotBank bank[kPoolBanks];
    int refs = 0;                        // contexts that used it
    std::vector<uint8_t *> retired;      // outgrown banks (freed with it)
};
static SlotPool g_pool[kMaxDevices];

static void
pool_release(int device, const qhuff_ctx *c)
{
    if (device < 0 || device >= kMaxDevices)
        return;
    SlotPool &sp = g_pool[device];
    std::lock_guard<std::mutex> g(sp.mu);
    for (SlotBank &b : sp.bank)
        if (b.last_ctx == c)             // (its launches have completed)
            b.last_ctx = nullptr;
    if (--sp.refs > 0)
        return;
    for (SlotBank &b : sp.bank)
    {
        if (b.p)
            (void) hipFree(b.p);
        if (b.ev)
            (void) hipEventDestroy(b.ev);
        b = SlotBank();
    }
    for (uint8_t *q : sp.retired)
        (void) hipFree(q);
    sp.retired.clear();
}

static uint64_t
max_grid_waves(const qhuff_ctx *c)
{
    const uint64_t e = (uint64_t) c->enc_grid * encode_waves_per_block();
    const uint64_t d = (uint64_t) c->dec_grid * decode_waves_per_block();
    return e > d ? e : d;
}

// the bank context c launches on (sp.mu held): its own; else a free one
// (never used, or its context closed); else, if c's bank was taken from it,
// a new one (up to c->max_banks); else the one c had, or bank 0
static uint32_t
pool_pick(SlotPool &sp, const qhuff_ctx *c)
{
    const uint32_t own = c->pool_bank;
    if (own && (sp.bank[own - 1].last_ctx == c || !sp.bank[own - 1].last_ctx))
        return own - 1;
    for (uint32_t i = 0; i < c->max_banks; ++i)
        if (sp.bank[i].p && !sp.bank[i].last_ctx)
            return i;
    if (own || !sp.bank[0].p)
        for (uint32_t i = 0; i < c->max_banks; ++i)
            if (!sp.bank[i].p)
                return i;
    return own ? own - 1 : 0;
}

// Runs launch(slots) for a launch of `grid` workgroups of `wpb` waves: the
// big-tile slots a full kernel needs (*full), null for the lean one.  When
// they cannot be allocated the launch runs the lean kernel (*full is
// cleared): big tiles out of line, the same output.
template <class F>
static int
with_slots(qhuff_ctx *c, uint32_t grid, uint64_t wpb, bool *full,
           hipStream_t st, F launch)
{
    if (!*full)
        return launch((uint8_t *) nullptr);
    if (grid <= kSmallGrid)
    {
        if (!c->big_small)
        {
            const uint64_t w = (uint64_t) kSmallGrid
                * (uint64_t) (encode_waves_per_block() > decode_waves_per_block()
                              ? encode_waves_per_block() : decode_waves_per_block());
            if (hipMalloc((void **) &c->big_small, w * kWaveSlotBytes) != hipSuccess)
            {
                c->big_small = nullptr;
                (void) hipGetLastError();
                *full = false;
                return launch((uint8_t *) nullptr);
            }
        }
        return launch(c->big_small);
    }
    if (c->device < 0 || c->device >= kMaxDevices)
    {
        *full = false;
        return launch((uint8_t *) nullptr);
    }
    SlotPool &sp = g_pool[c->device];
    std::lock_guard<std::mutex> g(sp.mu);
    if (!c->pool_ref)
    {
        ++sp.refs;
        c->pool_ref = true;
    }
    const uint64_t need = (uint64_t) grid * wpb;
    uint32_t bi = pool_pick(sp, c);
    if (!sp.bank[bi].p && bi != 0 && sp.bank[0].p)
    {
        // a new bank for a context whose bank was taken: if it cannot be
        // had, share (the ordering below), never the lean kernel
        const uint64_t mw = max_grid_waves(c);
        const uint64_t w = mw > need ? mw : need;
        if (hipMalloc((void **) &sp.bank[bi].p, w * kWaveSlotBytes) == hipSuccess)
            sp.bank[bi].waves = w;
        else
        {
            sp.bank[bi].p = nullptr;
            (void) hipGetLastError();
            bi = c->pool_bank ? c->pool_bank - 1 : 0;
        }
    }
    SlotBank &b = sp.bank[bi];
    if (b.waves < need)
    {
        if (b.p)
        {
            // (a grid larger than any seen: launches still running on the
            // old bank keep it until the pool's last user closes)
            sp.retired.push_back(b.p);
            b.p = nullptr;
            b.waves = 0;
        }
        const uint64_t mw = max_grid_waves(c);
        const uint64_t w = mw > need ? mw : need;
        if (hipMalloc((void **) &b.p, w * kWaveSlotBytes) != hipSuccess)
        {
            b.p = nullptr;
            (void) hipGetLastError();
            *full = false;
            return launch((uint8_t *) nullptr);
        }
        b.waves = w;
    }
    if (b.last_ctx && b.last_ctx != c)
    {
        // after the bank's last launch, another context's: everything on
        // its stream so far
        if (!b.ev)
            HIPCHK(c, hipEventCreateWithFlags(&b.ev, hipEventDisableTiming));
        hipError_t e = hipEventRecord(b.ev, b.last_st);
        if (e == hipSuccess)
            e = hipStreamWaitEvent(st, b.ev, 0);
        if (e != hipSuccess)
        {
            (void) hipGetLastError();
            HIPCHK(c, hipDeviceSynchronize());
        }
    }
    const int rc = launch(b.p);
    if (rc == QHUFF_OK)
    {
        b.last_ctx = c;
        b.last_st = st;
        c->pool_bank = bi + 1;
    }
    return rc;
}

extern "C" int
qhuff_open(int device, qhuff_ctx **ctx_out)
{
    if (!ctx_out)
        return QHUFF_EINVAL;
    *ctx_out = nullptr;
    int ndev = 0;
    if (hipGetDeviceCount(&ndev) != hipSuccess || device < 0 || device >= ndev)
        return QHUFF_ENODEV;
    hipDeviceProp_t prop;
    if (hipGetDeviceProperties(&prop, device) != hipSuccess)
        return QHUFF_ENODEV;
    if (strncmp(prop.gcnArchName, "gfx950", 6) != 0)
        return QHUFF_ENODEV;              // code objects are gfx950 only
    qhuff_ctx *c = new (std::nothrow) qhuff_ctx();
    if (!c)
        return QHUFF_ENOMEM;
    c->device = device;
    HIPCHK(c, hipSetDevice(device));
    c->n_cu = prop.multiProcessorCount;
    HostTables *ht = new HostTables;
    build_tables(ht);
    DevTables dt;
    for (int i = 0; i < 257; ++i)
        dt.enc[i] = make_uint2(ht->code[i], ht->bits[i]);
    memcpy(dt.win, ht->win, sizeof(dt.win));
    memcpy(dt.sorted, ht->sorted, sizeof(dt.sorted));
    memcpy(dt.long2, ht->long2, sizeof(dt.long2));
    memset(&c->lp, 0, sizeof(c->lp));
    c->lp.n = ht->n_long;
    memcpy(c->lp.l, ht->longc, sizeof(LongLen) * ht->n_long);
    delete ht;
    int rc, occ_e = 0, occ_d = 0, occ_h = 0;
    hipError_t e = encode_occupancy(&occ_e);
    if (e == hipSuccess)
        e = decode_occupancy(&occ_d);
    if (e == hipSuccess)
        e = hash_occupancy(&occ_h);
    if (e != hipSuccess || occ_e < 1 || occ_d < 1 || occ_h < 1)
    {
        char what[96];
        snprintf(what, sizeof(what), "occupancy query (enc %d dec %d hash %d)",
                 occ_e, occ_d, occ_h);
        rc = fail(c, e, what);
        delete c;
        return rc ? rc : QHUFF_EDEVICE;
    }
    // One launch's grid: the workgroups that fit at once (tiles come from
    // in-order tickets, so a grid that is not co-resident -- another
    // context or process on the GPU -- is slower, not wrong).
    c->enc_grid = (uint32_t) (occ_e * c->n_cu);
    c->dec_grid = (uint32_t) (occ_d * c->n_cu);
    c->hash_grid = (uint32_t) (occ_h * c->n_cu);
    e = hipMalloc((void **) &c->tab, sizeof(DevTables));
    if (e != hipSuccess)
    {
        rc = fail(c, e, "hipMalloc tables");
        delete c;
        return rc;
    }
    e = hipMemcpy(c->tab, &dt, sizeof(dt), hipMemcpyHostToDevice);
    if (e == hipSuccess)
        e = hipMalloc((void **) &c->err, kErrWords * sizeof(uint32_t));
    if (e == hipSuccess)
        e = hipMemset(c->err, 0, kErrWords * sizeof(uint32_t));
    if (e == hipSuccess)
    {
        const char *kv = getenv("QHUFF_KERNELS");
        c->kernels = !kv ? 0 : !strcmp(kv, "lean") ? 1 : !strcmp(kv, "full") ? 2 : 0;
    }
    if (e == hipSuccess)
        e = hipStreamCreateWithFlags(&c->own_stream, hipStreamNonBlocking);
    if (e == hipSuccess)
        e = hipEventCreateWithFlags(&c->ev_last, hipEventDisableTiming);
    if (e == hipSuccess)
        e = hipHostMalloc((void **) &c->err_host, 4 * sizeof(uint32_t),
                          hipHostMallocMapped | hipHostMallocCoherent);
    if (e == hipSuccess)
    {
        memset(c->err_host, 0, 4 * sizeof(uint32_t));
        e = hipHostGetDevicePointer((void **) &c->err_host_dev, c->err_host, 0);
    }
    if (e != hipSuccess)
    {
        rc = fail(c, e, "context setup");
        qhuff_close(c);
        return rc;
    }
    c->epoch = 0;
    c->hint[0] = c->hint[1] = -1;
    c->max_banks = kPoolBanks;
    if (const char *sb = getenv("QHUFF_SLOT_BANKS"))
    {
        const uint32_t k = (uint32_t) strtoul(sb, nullptr, 0);
        if (k >= 1 && k <= kPoolBanks)
            c->max_banks = k;
    }
    {
        // tuning override: fewer workgroups per CU than fit
        const char *g = getenv("QHUFF_GRID_WG_PER_CU");
        if (g)
        {
            uint32_t k = (uint32_t) strtoul(g, nullptr, 0);
            if (k >= 1 && k <= (uint32_t) occ_e)
                c->enc_grid = k * c->n_cu;
            if (k >= 1 && k <= (uint32_t) occ_d)
                c->dec_grid = k * c->n_cu;
        }
        // experiment: a percentage of the resident grid (half the CUs' worth
        // of workgroups at 50: per-CU vs chip-wide limits)
        const char *pc = getenv("QHUFF_GRID_PCT");
        if (pc)
        {
            const uint32_t q = (uint32_t) strtoul(pc, nullptr, 0);
            if (q >= 1 && q <= 100)
            {
                c->enc_grid = c->enc_grid * q / 100 ? c->enc_grid * q / 100 : 1;
                c->dec_grid = c->dec_grid * q / 100 ? c->dec_grid * q / 100 : 1;
            }
        }
    }
    *ctx_out = c;
    return QHUFF_OK;
}

extern "C" void
qhuff_close(qhuff_ctx *c)
{
    if (!c)
        return;
    (void) hipSetDevice(c->device);
    if (c->svc)
        qhuff_svc_close(c->svc);
    if (c->own_stream)
        (void) hipStreamSynchronize(c->own_stream);
    (void) hipDeviceSynchronize();
    if (c->tab)
        (void) hipFree(c->tab);
    if (c->flags)
        (void) hipFree(c->flags);
    if (c->big_small)
        (void) hipFree(c->big_small);
    if (c->pool_ref)
        pool_release(c->device, c);
    if (c->err)
        (void) hipFree(c->err);
    if (c->d_stage)
        (void) hipFree(c->d_stage);
    if (c->h_stage)
        (void) hipHostFree(c->h_stage);
    if (c->prof)
        (void) hipFree(c->prof);
    if (c->tev)
    {
        for (unsigned i = 0; i < 2 * QHUFF_TIMING_SLOTS; ++i)
            (void) hipEventDestroy(c->tev[i]);
        delete[] c->tev;
    }
    if (c->own_stream)
        (void) hipStreamDestroy(c->own_stream);
    if (c->ev_last)
        (void) hipEventDestroy(c->ev_last);
    if (c->err_host)
        (void) hipHostFree(c->err_host);
    if (c->pipe_ready)
    {
        (void) hipStreamDestroy(c->h2d_stream);
        (void) hipStreamDestroy(c->d2h_stream);
        for (unsigned i = 0; i < kMaxChunks; ++i)
        {
            (void) hipEventDestroy(c->ev_in[i]);
            (void) hipEventDestroy(c->ev_k[i]);
            (void) hipEventDestroy(c->ev_out[i]);
        }
    }
    delete c->pool;
    delete c;
}

extern "C" const char *
qhuff_last_error(qhuff_ctx *c)
{
    return c ? c->err_msg : t_open_err;
}

extern "C" int
qhuff_device_error(qhuff_ctx *c)
{
    if (!c)
        return QHUFF_EINVAL;
    HIPCHK(c, hipSetDevice(c->device));
    HIPCHK(c, hipDeviceSynchronize());
    uint32_t v = 0;
    HIPCHK(c, hipMemcpy(&v, c->err, 4, hipMemcpyDeviceToHost));
    if (v)
        HIPCHK(c, hipMemset(c->err, 0, 4));
    v |= c->err_host[0];
    c->err_host[0] = 0;
    return (int) v;
}

// Profile builds: copy the stamp buffer of the last launch (synchronous).
// Returns the number of u64 words available (0 in normal builds).
extern "C" uint64_t
qhuff_profile_read(qhuff_ctx *c, uint64_t *dst, uint64_t max_words)
{
    if (!c || !c->prof)
        return 0;
    (void) hipDeviceSynchronize();
    const uint64_t w = c->prof_words < max_words ? c->prof_words : max_words;
    if (dst && w)
        (void) hipMemcpy(dst, c->prof, w * 8, hipMemcpyDeviceToHost);
    return c->prof_words;
}

extern "C" uint64_t
qhuff_encode_bound(uint64_t in_bytes, uint32_t n, unsigned mode)
{
    // 30-bit longest code: ceil(30 * len / 8) per string; framing adds at
    // most 6 bytes of prefixed length (32-bit value) per literal
    uint64_t b = (in_bytes * 30 + 7) / 8 + n;
    if (mode)
        b += 6ull * n;
    return b + 16;
}

extern "C" uint64_t
qhuff_decode_bound(uint64_t in_bytes, uint32_t n)
{
    (void) n;
    return in_bytes * 8 / 5 + 16;
}

// look-back workspace: the tile tickets [2][kTickGroups] (u32, kTickStride
// apart), tile flags [cap_tiles], super flags [cap_super], super
// accumulators [2][cap_super] (u64, kAccStride apart)
constexpr size_t kTickBytes = 4 * 2 * kTickGroups * kTickStride;
static size_t
lb_bytes(uint64_t cap_tiles, uint64_t cap_super)
{
    return kTickBytes + 8 * (cap_tiles * kFlagStride + cap_super + 2 * cap_super * kAccStride);
}

// make room for the look-back workspace of `tiles` tiles and advance the
// epoch (flags are epoch-tagged; the claim counters and super accumulators
// of a launch are cleared by the launch before it).  Orders the launch
// after the context's previous one when that ran on another stream, and
// reports (then clears) a device error a previous launch left behind.
static int
prepare_launch(qhuff_ctx *c, uint64_t tiles, hipStream_t st)
{
    if (c->err_host[0])
    {
        snprintf(c->err_msg, sizeof(c->err_msg),
                 "device error %u in an earlier launch (outputs invalid)",
                 c->err_host[0]);
        c->err_host[0] = 0;
        (void) hipStreamSynchronize(c->last_stream);
        (void) hipMemset(c->err, 0, 4);
        return QHUFF_EDEVICE;
    }
    if (c->have_last && st != c->last_stream)
    {
        // everything queued on the previous stream so far, our last launch
        // included, before this one
        HIPCHK(c, hipEventRecord(c->ev_last, c->last_stream));
        HIPCHK(c, hipStreamWaitEvent(st, c->ev_last, 0));
    }
    if (tiles > c->cap_tiles)
    {
        if (c->flags)
        {
            HIPCHK(c, hipStreamSynchronize(st));
            HIPCHK(c, hipFree(c->flags));
            c->flags = nullptr;
        }
        uint64_t cap = tiles < 4096 ? 4096 : tiles;
        uint64_t caps = (cap + kSuper - 1) / kSuper;
        HIPCHK(c, hipMalloc((void **) &c->flags, lb_bytes(cap, caps)));
        HIPCHK(c, hipMemsetAsync(c->flags, 0, lb_bytes(cap, caps), st));
        c->cap_tiles = cap;
        c->cap_super = caps;
    }
    c->epoch = (c->epoch + 1) & kEpochMask;
    if (c->epoch == 0)
    {
        // wrapped: stale flags could alias the new epoch, and the
        // accumulators of epoch 1 were last used, not cleared
        HIPCHK(c, hipMemsetAsync(c->flags, 0, lb_bytes(c->cap_tiles, c->cap_super),
                                 st));
        c->epoch = 1;
    }
    return QHUFF_OK;
}

// after a look-back launch on st (the ordering event is recorded only when
// a later launch comes on another stream, see prepare_launch)
static int
finish_launch(qhuff_ctx *c, hipStream_t st)
{
    c->last_stream = st;
    c->have_last = true;
    return QHUFF_OK;
}

static Coord
coord(qhuff_ctx *c, uint64_t tiles)
{
    Coord k;
    k.prof = nullptr;
#ifdef QHUFF_PROFILE
    {
        const size_t words = (size_t) c->n_cu * 32 * kProfIters * kProfSlots;
        if (!c->prof && hipMalloc((void **) &c->prof, words * 8) == hipSuccess)
            c->prof_words = words;
        if (c->prof)
            (void) hipMemset(c->prof, 0, c->prof_words * 8);
        k.prof = c->prof;
    }
#endif
    k.tick = (uint32_t *) c->flags;
    k.flags = c->flags + kTickBytes / 8;
    k.sflags = k.flags + c->cap_tiles * kFlagStride;
    k.sacc = k.sflags + c->cap_super;
    k.cap_super = (uint32_t) c->cap_super;
    k.err = c->err;
    k.err_host = c->err_host_dev;
    k.epoch = c->epoch;
    k.n_tiles = (uint32_t) tiles;
    k.spread = 0;
    k.big = nullptr;                     // (with_slots)
    return k;
}

// the event pair of the next launch (kind QHUFF_KIND_*) with timing on, and
// its ring slot; *e0 = *e1 = null and kNoTiming otherwise.  The slot is
// taken by timing_commit once the launch has gone out: a launch that fails
// leaves no slot with unrecorded events behind.
constexpr uint32_t kNoTiming = 0xffffffffu;
static uint32_t
timing_slot(qhuff_ctx *c, uint32_t kind, hipEvent_t *e0, hipEvent_t *e1)
{
    *e0 = *e1 = nullptr;
    if (!c->t_on)
        return kNoTiming;
    // sampled: each timed launch costs the step ~4.6 us of queue time
    // (tools/timing_cost.py: 114.8 vs 105.6 us per encode + decode step)
    if (c->t_seen[kind]++ % c->t_every != 0)
        return kNoTiming;
    const uint32_t k = (uint32_t) (c->t_next % QHUFF_TIMING_SLOTS);
    *e0 = c->tev[2 * k];
    *e1 = c->tev[2 * k + 1];
    return k;
}

static void
timing_commit(qhuff_ctx *c, uint32_t k, uint32_t kind)
{
    if (k == kNoTiming)
        return;
    c->t_kind[k] = (uint8_t) kind;
    ++c->t_next;
}

extern "C" int
qhuff_timing_enable(qhuff_ctx *c, int on)
{
    if (!c)
        return QHUFF_EINVAL;
    HIPCHK(c, hipSetDevice(c->device));
    if (on && !c->tev)
    {
        hipEvent_t *ev = new (std::nothrow) hipEvent_t[2 * QHUFF_TIMING_SLOTS]();
        if (!ev)
            return QHUFF_ENOMEM;
        for (unsigned i = 0; i < 2 * QHUFF_TIMING_SLOTS; ++i)
        {
            const hipError_t e = hipEventCreate(&ev[i]);
            if (e != hipSuccess)
            {
                for (unsigned j = 0; j < i; ++j)
                    (void) hipEventDestroy(ev[j]);
                delete[] ev;
                return fail(c, e, "hipEventCreate (timing)");
            }
        }
        c->tev = ev;
    }
    c->t_on = on > 0;
    c->t_every = on > 1 ? (uint32_t) on : 1u;
    c->t_seen[0] = c->t_seen[1] = c->t_seen[2] = 0;
    c->t_first = c->t_next;
    return QHUFF_OK;
}

extern "C" int
qhuff_timing_read(qhuff_ctx *c, uint32_t *kind, double *us, uint32_t max)
{
    if (!c || (max && (!kind || !us)))
        return QHUFF_EINVAL;
    if (!c->tev)
        return 0;
    HIPCHK(c, hipSetDevice(c->device));
    uint64_t a = c->t_first;
    const uint64_t b = c->t_next;
    if (b - a > QHUFF_TIMING_SLOTS)
        a = b - QHUFF_TIMING_SLOTS;
    if (b - a > max)
        a = b - max;
    uint32_t n = 0;
    for (uint64_t i = a; i < b; ++i, ++n)
    {
        const uint32_t k = (uint32_t) (i % QHUFF_TIMING_SLOTS);
        HIPCHK(c, hipEventSynchronize(c->tev[2 * k + 1]));
        float ms = 0.f;
        HIPCHK(c, hipEventElapsedTime(&ms, c->tev[2 * k], c->tev[2 * k + 1]));
        kind[n] = c->t_kind[k];
        us[n] = 1e3 * (double) ms;
    }
    c->t_first = b;
    return (int) n;
}

// Workgroups for a launch of `tiles` tiles, at most `cap` (the co-resident
// count: more would only queue); tiles are claimed from tickets, so any grid
// size is correct.  A batch of at most one tile per wave of the full grid
// is spread: one workgroup per tile up to `cap`, the first *spread waves
// of each taking one tile each (Coord::spread; fewer waves per CU code
// their tile faster, and the whole batch is handed out by one returning
// add per workgroup on one counter, in order).  Larger batches: every wave,
// ticket groups.
static uint32_t
grid_for(const qhuff_ctx *c, uint64_t tiles, uint64_t waves_per_block,
         uint32_t cap, uint32_t *spread)
{
    (void) c;
    *spread = 0;
    if (tiles <= (uint64_t) cap * waves_per_block)
    {
        const uint32_t g = (uint32_t) (tiles < cap ? tiles : cap);
        *spread = (uint32_t) ((tiles + g - 1) / g);
        return g;
    }
    const uint64_t need = (tiles + waves_per_block - 1) / waves_per_block;
    return (uint32_t) (need < cap ? need : cap);
}

// The kernel variant of the next launch of `kind` (0 encode, 1 decode).
// The full kernel codes every batch at its best; the lean one (no big-tile
// slots, no cooperative long-string decode: those tiles out of line, one
// lane per string, up to 30x slower on the QIF corpus) is 0.7 % (encode) /
// 1.3 % (decode) faster on batches that never need them (profiles/r06_i,
// same-box pairs).  So: the full kernel, unless the caller's batch is known
// to have no string over 128 bytes and no tile over the 3 KB stage -- the
// host-memory calls read their offsets (host_hint), a device-pointer caller
// may say so with qhuff_batch_hint -- or QHUFF_KERNELS pins one.  (Until
// round 5 decode went by a history of earlier launches, lean until one
// reported such tiles: the first launch of a long-string batch after token
// batches then took 4.3x its warmed time.  Round 6 took the full decode
// kernel's cost on the token batch from +3.3 % to +1.3 %: the lane id
// opaque to the optimiser, uniform flags as u32, the cooperative phase on
// the big-tile path)
static bool
pick_full(qhuff_ctx *c, int kind)
{
    // a hint applies to the next launch of its kind only, whatever decides
    // this one
    const int hint = c->hint[kind];
    c->hint[kind] = -1;
    if (c->kernels)
        return c->last_full[kind] = c->kernels == 2;
    if (hint >= 0)
        return c->last_full[kind] = hint > 0;
    return c->last_full[kind] = true;
}

extern "C" int
qhuff_kernel_variant(qhuff_ctx *c, int kind)
{
    if (!c || (kind != QHUFF_KIND_ENCODE && kind != QHUFF_KIND_DECODE))
        return QHUFF_EINVAL;
    return c->last_full[kind] ? 1 : 0;
}

extern "C" int
qhuff_encode_batch(qhuff_ctx *c, const uint8_t *in, const uint32_t *in_off,
                   uint32_t n, unsigned mode, uint8_t *out, uint32_t *out_off,
                   void *stream)
{
    if (!c || !in_off || !out_off || (n && (!in || !out)))
        return QHUFF_EINVAL;
    if (mode != 0 && mode != 3 && mode != 5 && mode != 7)
        return QHUFF_EINVAL;
    hipStream_t st = (hipStream_t) stream;
    HIPCHK(c, hipSetDevice(c->device));
    if (n == 0)
    {
        HIPCHK(c, hipMemsetAsync(out_off, 0, 4, st));
        return QHUFF_OK;
    }
    uint64_t tiles = (n + kWT - 1) / kWT;
    int rc = prepare_launch(c, tiles, st);
    if (rc)
        return rc;
    EncArgs a;
    a.in = in;
    a.in_off = in_off;
    a.out = out;
    a.out_off = out_off;
    a.enc = c->tab->enc;
    a.n = n;
    a.mode = mode;
    a.c = coord(c, tiles);
    const uint64_t wpb = (uint64_t) encode_waves_per_block();
    const uint32_t grid = grid_for(c, tiles, wpb, c->enc_grid, &a.c.spread);
    bool full = pick_full(c, 0);
    rc = with_slots(c, grid, wpb, &full, st, [&](uint8_t *slots) -> int {
        a.c.big = slots;
        hipEvent_t e0, e1;
        const uint32_t ts = timing_slot(c, QHUFF_KIND_ENCODE, &e0, &e1);
        HIPCHK(c, launch_encode(a, grid, st, e0, e1, full));
        timing_commit(c, ts, QHUFF_KIND_ENCODE);
        return QHUFF_OK;
    });
    if (rc)
        return rc;
    c->last_full[0] = full;
    return finish_launch(c, st);
}

extern "C" int
qhuff_decode_batch(qhuff_ctx *c, const uint8_t *in, const uint32_t *in_off,
                   uint32_t n, uint8_t *out, uint32_t *out_off,
                   uint8_t *status, void *stream)
{
    if (!c || !in_off || !out_off || (n && (!in || !out || !status)))
        return QHUFF_EINVAL;
    hipStream_t st = (hipStream_t) stream;
    HIPCHK(c, hipSetDevice(c->device));
    if (n == 0)
    {
        HIPCHK(c, hipMemsetAsync(out_off, 0, 4, st));
        return QHUFF_OK;
    }
    const uint64_t ts = decode_tile_strings();
    uint64_t tiles = (n + ts - 1) / ts;
    int rc = prepare_launch(c, tiles, st);
    if (rc)
        return rc;
    DecArgs a;
    a.in = in;
    a.in_off = in_off;
    a.out = out;
    a.out_off = out_off;
    a.status = status;
    a.win = c->tab->win;
    a.sorted = c->tab->sorted;
    a.long2 = c->tab->long2;
    a.n = n;
    a.c = coord(c, tiles);
    a.lp = c->lp;
    const uint64_t wpb = (uint64_t) decode_waves_per_block();
    const uint32_t grid = grid_for(c, tiles, wpb, c->dec_grid, &a.c.spread);
    // (keep: the per-string replay -- the lean keep kernel, never timed, and
    // outside the variant choice of the batch kernel: ADVICE r04)
    bool full = false;
    if (!c->keep_rejected)
        full = pick_full(c, 1);
    else
        c->hint[1] = -1;                 // (consumed by this launch too)
    rc = with_slots(c, grid, wpb, &full, st, [&](uint8_t *slots) -> int {
        a.c.big = slots;
        hipEvent_t e0 = nullptr, e1 = nullptr;
        const uint32_t ts = c->keep_rejected
            ? kNoTiming : timing_slot(c, QHUFF_KIND_DECODE, &e0, &e1);
        HIPCHK(c, launch_decode(a, grid, st, e0, e1, c->keep_rejected, full));
        timing_commit(c, ts, QHUFF_KIND_DECODE);
        return QHUFF_OK;
    });
    if (rc)
        return rc;
    if (!c->keep_rejected)
        c->last_full[1] = full;
    return finish_launch(c, st);
}

// ---- header hashing ---------------------------------------------------------

static int
hash_call(qhuff_ctx *c, const uint8_t *in, const uint32_t *off, uint32_t n,
          uint32_t seed, uint32_t *h1, uint32_t *h2, bool pairs, void *stream)
{
    if (!c || !off || (n && (!in || !h1 || (pairs && !h2))))
        return QHUFF_EINVAL;
    if (pairs && n > 0x7fffffffu)
        return QHUFF_ERANGE;
    HIPCHK(c, hipSetDevice(c->device));
    if (n == 0)
        return QHUFF_OK;
    HashArgs a;
    a.in = in;
    a.off = off;
    a.h1 = h1;
    a.h2 = h2;
    a.n = n;
    a.seed = seed;
    a.pairs = pairs ? 1u : 0u;
    hipEvent_t e0, e1;
    const uint32_t ts = timing_slot(c, QHUFF_KIND_HASH, &e0, &e1);
    HIPCHK(c, launch_hash(a, c->hash_grid, (hipStream_t) stream, e0, e1));
    timing_commit(c, ts, QHUFF_KIND_HASH);
    return QHUFF_OK;
}

extern "C" int
qhuff_xxh32_headers(qhuff_ctx *c, const uint8_t *in, const uint32_t *off,
                    uint32_t n, uint32_t seed, uint32_t *name_hash,
                    uint32_t *nameval_hash, void *stream)
{
    return hash_call(c, in, off, n, seed, name_hash, nameval_hash, true,
                     stream);
}

extern "C" int
qhuff_xxh32_batch(qhuff_ctx *c, const uint8_t *in, const uint32_t *in_off,
                  uint32_t n, uint32_t seed, uint32_t *hash, void *stream)
{
    return hash_call(c, in, in_off, n, seed, hash, nullptr, false, stream);
}

// ---- host-memory path ------------------------------------------------------

static int
ensure_stage(qhuff_ctx *c, size_t bytes)
{
    if (bytes > c->h_stage_cap)
    {
        if (c->h_stage)
            (void) hipHostFree(c->h_stage);
        c->h_stage = nullptr;
        c->h_stage_cap = 0;
        HIPCHK(c, hipHostMalloc((void **) &c->h_stage, bytes));
        c->h_stage_cap = bytes;
    }
    if (bytes > c->d_stage_cap)
    {
        if (c->d_stage)
            (void) hipFree(c->d_stage);
        c->d_stage = nullptr;
        c->d_stage_cap = 0;
        HIPCHK(c, hipMalloc((void **) &c->d_stage, bytes));
        c->d_stage_cap = bytes;
    }
    return QHUFF_OK;
}

static inline size_t
up16(size_t x)
{
    return (x + 15) & ~(size_t) 15;
}

// The kernels' sticky error word, read from its pinned host mirror (the
// kernels set both; call once the launch's stream has been synchronised):
// no device round trip on the synchronous paths.
static int
mirror_error(qhuff_ctx *c)
{
    const uint32_t v = __atomic_exchange_n(&c->err_host[0], 0u, __ATOMIC_ACQ_REL);
    if (!v)
        return QHUFF_OK;
    (void) hipMemset(c->err, 0, 4);
    snprintf(c->err_msg, sizeof(c->err_msg), "device error %u", v);
    return QHUFF_EDEVICE;
}

static int
pipe_setup(qhuff_ctx *c)
{
    if (c->pipe_ready)
        return QHUFF_OK;
    HIPCHK(c, hipStreamCreateWithFlags(&c->h2d_stream, hipStreamNonBlocking));
    HIPCHK(c, hipStreamCreateWithFlags(&c->d2h_stream, hipStreamNonBlocking));
    for (unsigned i = 0; i < kMaxChunks; ++i)
    {
        HIPCHK(c, hipEventCreateWithFlags(&c->ev_in[i], hipEventDisableTiming));
        HIPCHK(c, hipEventCreateWithFlags(&c->ev_k[i], hipEventDisableTiming));
        HIPCHK(c, hipEventCreateWithFlags(&c->ev_out[i], hipEventDisableTiming));
    }
    unsigned t = 8;
    if (const char *e = getenv("QHUFF_HOST_THREADS"))
        t = (unsigned) strtoul(e, nullptr, 0);
    if (t > 64)
        t = 64;
    c->pool = new CopyPool(t > 1 ? t - 1 : 0);   // + the calling thread
    c->pipe_ready = true;
    return QHUFF_OK;
}

// The variant the kernels' own rules call for on a batch whose offsets the
// host holds (the host-memory paths): the full kernel when a string is
// longer than kHintLen bytes (decode: the cooperative threshold, kCoopMin
// Huffman bytes; encode: a payload the full emit copies with the whole
// wave, at ~8 bits a byte) or a 64-string tile spans more than the 3 KB
// stage can take (a big tile).  One pass over the offsets on the copy
// workers.  VERDICT r04 item 2: the device-pointer calls can only go by
// history; these need not.
constexpr uint32_t kHintLen = 128;
constexpr uint32_t kHintSpan = 3072 - 32;
static bool
host_rare(qhuff_ctx *c, const uint32_t *off, uint32_t n)
{
    std::atomic<bool> rare{false};
    const uint32_t tiles = (n + 63) / 64, per = 1024;   // tiles per slice
    c->pool->run((tiles + per - 1) / per, [&](unsigned k) {
        const uint32_t t0 = k * per, t1 = t0 + per < tiles ? t0 + per : tiles;
        bool r = false;
        for (uint32_t t = t0; t < t1 && !r; ++t)
        {
            const uint32_t a = 64 * t, b = a + 64 < n ? a + 64 : n;
            r = off[b] - off[a] > kHintSpan;
            for (uint32_t i = a; i < b; ++i)
                r |= off[i + 1] - off[i] > kHintLen;
        }
        if (r)
            rare.store(true, std::memory_order_relaxed);
    });
    return rare.load();
}

static void
host_hint(qhuff_ctx *c, bool enc, const uint32_t *off, uint32_t n)
{
    if (c->kernels == 0)
        c->hint[enc ? 0 : 1] = host_rare(c, off, n) ? 1 : 0;
}

extern "C" int
qhuff_batch_hint(qhuff_ctx *c, int kind, int hint)
{
    if (!c || (kind != QHUFF_KIND_ENCODE && kind != QHUFF_KIND_DECODE)
            || hint < -1 || hint > 1)
        return QHUFF_EINVAL;
    c->hint[kind] = hint;
    return QHUFF_OK;
}

extern "C" int
qhuff_batch_needs_full(const uint32_t *off, uint32_t n)
{
    if (!off)
        return QHUFF_EINVAL;
    for (uint32_t a = 0; a < n; a += 64)
    {
        const uint32_t b = a + 64 < n ? a + 64 : n;
        if (off[b] - off[a] > kHintSpan)
            return 1;
        for (uint32_t i = a; i < b; ++i)
            if (off[i + 1] - off[i] > kHintLen)
                return 1;
    }
    return 0;
}

// The PCIe-inclusive path as a chunked pipeline.  The batch is cut into K
// string ranges; per chunk: pinned staging copy (copy workers) -> H2D on the
// upload stream -> kernel on the context stream (its out_off / status come
// back on the same stream) -> once the chunk's size is known, D2H of exactly
// its output bytes on the download stream -> copy out + rebase out_off on
// the host.  Chunk i's host copies overlap chunk i-1's kernel and transfers.
// Kernels stay serialised on one stream (one look-back workspace).
//
// Stage layout (pinned and device alike): [in bytes | in_off (n + 1) |
// out: per-chunk bound regions | out_off: n_i + 1 per chunk | status n].
// The kernels read the original offsets: `in` is passed rebased by -in_off[0].
//
// Shard k of a multi-context call (qhuff_*_batch_host_multi, `sync`): the
// shard's output goes to `out` at a base only known once every earlier shard
// has sized its output, so its copies out of the pinned stage wait until
// all its chunks are fetched and the base is published -- its uploads,
// kernels and downloads never wait for another shard.
struct ShardSync
{
    std::mutex mu;
    std::condition_variable cv;
    std::vector<uint64_t> total;         // output bytes of each shard
    std::vector<char> known;
    bool failed = false;
    explicit ShardSync(unsigned g) : total(g, 0), known(g, 0) {}
    void publish(unsigned k, uint64_t t)
    {
        std::lock_guard<std::mutex> l(mu);
        total[k] = t;
        known[k] = 1;
        cv.notify_all();
    }
    void fail()
    {
        std::lock_guard<std::mutex> l(mu);
        failed = true;
        cv.notify_all();
    }
    // the output bytes of shards [0, k), or ~0 if one of them failed
    uint64_t base_of(unsigned k)
    {
        std::unique_lock<std::mutex> l(mu);
        uint64_t b = 0;
        for (unsigned j = 0; j < k; ++j)
        {
            cv.wait(l, [&] { return known[j] || failed; });
            if (failed)
                return ~0ull;
            b += total[j];
        }
        return b;
    }
};

// ---- caller buffers registered for direct DMA (qhuff_host_register) -------
//
// The host path stages the caller's input into pinned memory and its output
// back out of it: ~67 MB of host memcpy for a 1M-string encode + decode,
// which bounds it near the copy workers' rate (~22 GB/s of payload each way,
// DESIGN.md section 5).  Buffers the caller registered once (hipHostRegister,
// portable: every device's DMA engines reach them) are read and written by
// the transfers directly: no staging copy, and the path is bound by PCIe.
struct HostReg
{
    std::mutex mu;
    std::vector<std::pair<uintptr_t, uintptr_t>> r;      // [begin, end)
};
static HostReg g_reg;

static bool
host_registered(const void *p, uint64_t bytes)
{
    if (!bytes)
        return true;
    const uintptr_t a = (uintptr_t) p, b = a + bytes;
    std::lock_guard<std::mutex> g(g_reg.mu);
    for (const auto &x : g_reg.r)
        if (x.first <= a && b <= x.second)
            return true;
    return false;
}

extern "C" int
qhuff_host_register(void *ptr, size_t bytes)
{
    if (!ptr || !bytes)
        return QHUFF_EINVAL;
    std::lock_guard<std::mutex> g(g_reg.mu);
    for (const auto &x : g_reg.r)
        if (x.first == (uintptr_t) ptr)
            return QHUFF_EINVAL;         // (already registered)
    const hipError_t e = hipHostRegister(ptr, bytes, hipHostRegisterPortable);
    if (e != hipSuccess)
    {
        (void) hipGetLastError();
        snprintf(t_open_err, sizeof(t_open_err), "hipHostRegister: %s",
                 hipGetErrorString(e));
        return e == hipErrorOutOfMemory ? QHUFF_ENOMEM : QHUFF_EDEVICE;
    }
    g_reg.r.emplace_back((uintptr_t) ptr, (uintptr_t) ptr + bytes);
    return QHUFF_OK;
}

extern "C" int
qhuff_host_unregister(void *ptr)
{
    std::lock_guard<std::mutex> g(g_reg.mu);
    for (size_t i = 0; i < g_reg.r.size(); ++i)
        if (g_reg.r[i].first == (uintptr_t) ptr)
        {
            const hipError_t e = hipHostUnregister(ptr);
            g_reg.r.erase(g_reg.r.begin() + (ptrdiff_t) i);
            if (e != hipSuccess)
            {
                (void) hipGetLastError();
                return QHUFF_EDEVICE;
            }
            return QHUFF_OK;
        }
    return QHUFF_EINVAL;
}

static int
host_batch(qhuff_ctx *c, bool enc, const uint8_t *in, const uint32_t *in_off,
           uint32_t n, unsigned mode, uint8_t *out, uint32_t *out_off,
           uint8_t *status, ShardSync *sync = nullptr, unsigned shard = 0,
           bool last_shard = true)
{
    if (!c || !in_off || !out_off || (n && (!in || !out)) || (!enc && n && !status))
        return QHUFF_EINVAL;
    HIPCHK(c, hipSetDevice(c->device));
    int rc = pipe_setup(c);
    if (rc)
        return rc;
    const uint64_t a0 = in_off[0], in_bytes = (uint64_t) in_off[n] - a0;
    // chunks of >= 2^chunk_shift bytes of input (QHUFF_HOST_CHUNK_SHIFT;
    // default 8 MB: measured on MI355X, 1M strings, 8 copy threads -- 2 MB
    // chunks 2.9 / 2.7 ms enc / dec, 4 MB 2.2 / 2.0, 8 MB 1.8 / 1.7, 16 MB
    // 1.9 / 2.3; tools/host_path_probe.py), at most kMaxChunks
    static const unsigned chunk_shift = [] {
        const char *e = getenv("QHUFF_HOST_CHUNK_SHIFT");
        const unsigned v = e ? (unsigned) strtoul(e, nullptr, 0) : 23u;
        return v >= 16 && v <= 30 ? v : 23u;
    }();
    unsigned K = (unsigned) (in_bytes >> chunk_shift);
    K = K < 1 ? 1 : (K > kMaxChunks ? kMaxChunks : K);
    if (K > n)
        K = n ? n : 1;
    uint32_t cut[kMaxChunks + 1];
    uint64_t ob[kMaxChunks + 1];                 // out region starts
    ob[0] = 0;
    for (unsigned i = 0; i <= K; ++i)
        cut[i] = (uint32_t) ((uint64_t) n * i / K);
    for (unsigned i = 0; i < K; ++i)
    {
        const uint32_t s0 = cut[i], s1 = cut[i + 1];
        const uint64_t b = (uint64_t) in_off[s1] - in_off[s0];
        ob[i + 1] = ob[i] + up16(enc ? qhuff_encode_bound(b, s1 - s0, mode)
                                     : qhuff_decode_bound(b, s1 - s0));
    }
    if (ob[K] > 0xffffffffull)
        return QHUFF_ERANGE;
    const size_t o_in = 0, o_off = up16(in_bytes);
    const size_t o_out = o_off + up16(4ull * (n + 1));
    const size_t o_oo = o_out + ob[K];
    const size_t o_st = o_oo + up16(4ull * (n + K));
    const size_t total = o_st + up16(n ? n : 1);
    rc = ensure_stage(c, total);
    if (rc)
        return rc;
    uint8_t *H = c->h_stage, *D = c->d_stage;
    hipStream_t sk = c->own_stream;
    uint64_t base = 0;                           // output bytes so far
    uint32_t tot[kMaxChunks];
    uint64_t obase[kMaxChunks];                  // chunk i's output start
    uint64_t fbase = 0;                          // (relative to the call's)
    // a small batch brings its whole output bound back right behind the
    // kernel: one synchronisation instead of two (latency, not bandwidth)
    const bool small = K == 1 && ob[1] <= (4u << 20);
    // caller buffers registered for DMA (qhuff_host_register): transferred
    // directly, no staging copy
    const bool din = host_registered(in + a0, in_bytes)
                  && host_registered(in_off, 4ull * (n + 1));
    const bool dout = !small
        && host_registered(out, enc ? qhuff_encode_bound(in_bytes, n, mode)
                                    : qhuff_decode_bound(in_bytes, n))
        && host_registered(out_off, 4ull * (n + 1))
        && (enc || host_registered(status, n));

    auto stage_in = [&](unsigned i) -> int {
        const uint32_t s0 = cut[i], s1 = cut[i + 1];
        const uint64_t b0 = in_off[s0] - a0, b1 = in_off[s1] - a0;
        const uint8_t *src_in = in + a0;
        const uint8_t *src_off = (const uint8_t *) in_off;
        if (!din)
        {
            c->pool->copy(H + o_in + b0, in + a0 + b0, b1 - b0);
            memcpy(H + o_off + 4ull * s0, in_off + s0, 4ull * (s1 - s0 + 1));
            src_in = H + o_in;
            src_off = H + o_off;
        }
        HIPCHK(c, hipMemcpyAsync(D + o_in + b0, src_in + b0, b1 - b0,
                                 hipMemcpyHostToDevice, c->h2d_stream));
        HIPCHK(c, hipMemcpyAsync(D + o_off + 4ull * s0, src_off + 4ull * s0,
                                 4ull * (s1 - s0 + 1), hipMemcpyHostToDevice,
                                 c->h2d_stream));
        HIPCHK(c, hipEventRecord(c->ev_in[i], c->h2d_stream));
        HIPCHK(c, hipStreamWaitEvent(sk, c->ev_in[i], 0));
        const uint8_t *din = D + o_in - a0;      // kernels see original offsets
        const uint32_t *doff = (const uint32_t *) (D + o_off) + s0;
        uint32_t *doo = (uint32_t *) (D + o_oo) + s0 + i;
        host_hint(c, enc, in_off + s0, s1 - s0);
        int r = enc ? qhuff_encode_batch(c, din, doff, s1 - s0, mode,
                                         D + o_out + ob[i], doo, sk)
                    : qhuff_decode_batch(c, din, doff, s1 - s0,
                                         D + o_out + ob[i], doo, D + o_st + s0,
                                         sk);
        if (r)
            return r;
        if (dout)
        {
            // the chunk-local offsets straight into out_off (rebased in
            // place by unstage), the chunk's total into the stage
            HIPCHK(c, hipMemcpyAsync(out_off + s0, doo, 4ull * (s1 - s0),
                                     hipMemcpyDeviceToHost, sk));
            HIPCHK(c, hipMemcpyAsync(H + o_oo + 4ull * (s1 + i), doo + (s1 - s0),
                                     4, hipMemcpyDeviceToHost, sk));
            if (!enc)
                HIPCHK(c, hipMemcpyAsync(status + s0, D + o_st + s0, s1 - s0,
                                         hipMemcpyDeviceToHost, sk));
        }
        else
        {
            HIPCHK(c, hipMemcpyAsync(H + o_oo + 4ull * (s0 + i), doo,
                                     4ull * (s1 - s0 + 1), hipMemcpyDeviceToHost,
                                     sk));
            if (!enc)
                HIPCHK(c, hipMemcpyAsync(H + o_st + s0, D + o_st + s0, s1 - s0,
                                         hipMemcpyDeviceToHost, sk));
        }
        if (small)
            HIPCHK(c, hipMemcpyAsync(H + o_out, D + o_out, ob[1],
                                     hipMemcpyDeviceToHost, sk));
        HIPCHK(c, hipEventRecord(c->ev_k[i], sk));
        return QHUFF_OK;
    };
    // chunk i's output bytes back: to the stage, or (dout) straight to
    // out + dst (once its base is known)
    auto issue_out = [&](unsigned i, uint64_t dst) -> int {
        HIPCHK(c, hipStreamWaitEvent(c->d2h_stream, c->ev_k[i], 0));
        if (tot[i])
            HIPCHK(c, hipMemcpyAsync(dout ? out + dst : H + o_out + ob[i],
                                     D + o_out + ob[i], tot[i],
                                     hipMemcpyDeviceToHost, c->d2h_stream));
        HIPCHK(c, hipEventRecord(c->ev_out[i], c->d2h_stream));
        return QHUFF_OK;
    };
    auto fetch = [&](unsigned i) -> int {
        HIPCHK(c, hipEventSynchronize(c->ev_k[i]));
        const uint32_t s1 = cut[i + 1];
        tot[i] = ((const uint32_t *) (H + o_oo))[s1 + i];
        obase[i] = fbase;
        fbase += tot[i];
        if (small)
            return QHUFF_OK;                     // already here
        // (a shard of a multi-context call learns its base only later: its
        // direct copies out wait for it)
        if (dout && sync)
            return QHUFF_OK;
        return issue_out(i, obase[i]);
    };
    auto unstage = [&](unsigned i) -> int {
        if (!small)
            HIPCHK(c, hipEventSynchronize(c->ev_out[i]));
        const uint32_t s0 = cut[i], s1 = cut[i + 1];
        if (dout)
        {
            // bytes and statuses are in place; the offsets get the base
            const uint32_t bs = (uint32_t) base;
            const uint32_t m = s1 - s0, sl = 1u << 16;
            if (bs)
                c->pool->run((m + sl - 1) / sl, [=](unsigned k) {
                    const uint32_t a = k * sl, b = a + sl < m ? a + sl : m;
                    for (uint32_t j = a; j < b; ++j)
                        out_off[s0 + j] += bs;
                });
            base += tot[i];
            return QHUFF_OK;
        }
        c->pool->copy(out + base, H + o_out + ob[i], tot[i]);
        const uint32_t *ho = (const uint32_t *) (H + o_oo) + s0 + i;
        const uint32_t bs = (uint32_t) base;
        const uint32_t m = s1 - s0, sl = 1u << 16;
        c->pool->run((m + sl - 1) / sl, [=](unsigned k) {
            const uint32_t a = k * sl, b = a + sl < m ? a + sl : m;
            for (uint32_t j = a; j < b; ++j)
                out_off[s0 + j] = bs + ho[j];
        });
        if (!enc)
            memcpy(status + s0, H + o_st + s0, m);
        base += tot[i];
        return QHUFF_OK;
    };

    if (n == 0)
    {
        if (sync)
        {
            sync->publish(shard, 0);
            base = sync->base_of(shard);
            if (base == ~0ull)
                return QHUFF_EDEVICE;
        }
        if (last_shard)
            out_off[0] = (uint32_t) base;
        return QHUFF_OK;
    }
    if (sync)
    {
        // every chunk in flight first, then the copies out at the base
        for (unsigned i = 0; i < K; ++i)
        {
            if ((rc = stage_in(i)))
                return rc;
            if (i >= 1 && (rc = fetch(i - 1)))
                return rc;
        }
        if ((rc = fetch(K - 1)))
            return rc;
        uint64_t t = 0;
        for (unsigned i = 0; i < K; ++i)
            t += tot[i];
        sync->publish(shard, t);
        base = sync->base_of(shard);
        if (base == ~0ull)
            return QHUFF_EDEVICE;
        if (dout && !small)
            for (unsigned i = 0; i < K; ++i)
                if ((rc = issue_out(i, base + obase[i])))
                    return rc;
        for (unsigned i = 0; i < K; ++i)
            if ((rc = unstage(i)))
                return rc;
    }
    else
    {
        for (unsigned i = 0; i < K; ++i)
        {
            if ((rc = stage_in(i)))
                return rc;
            if (i >= 1 && (rc = fetch(i - 1)))
                return rc;
            if (i >= 2 && (rc = unstage(i - 2)))
                return rc;
        }
        if ((rc = fetch(K - 1)))
            return rc;
        for (unsigned i = K >= 2 ? K - 2 : 0; i < K; ++i)
            if ((rc = unstage(i)))
                return rc;
    }
    // (a shard's closing offset is the next shard's first one: written by
    // the last shard only)
    if (last_shard)
        out_off[n] = (uint32_t) base;
    {
        if ((rc = mirror_error(c)))
            return rc;
    }
    return QHUFF_OK;
}

static bool svc_fits(const uint32_t *in_off, uint32_t n);
static int svc_call(qhuff_svc *v, bool enc, const uint8_t *in,
                    const uint32_t *in_off, uint32_t n, unsigned mode,
                    uint8_t *out, uint32_t *out_off, uint8_t *status);

extern "C" int
qhuff_encode_batch_host(qhuff_ctx *c, const uint8_t *in,
                        const uint32_t *in_off, uint32_t n, unsigned mode,
                        uint8_t *out, uint32_t *out_off)
{
    if (mode != 0 && mode != 3 && mode != 5 && mode != 7)
        return QHUFF_EINVAL;
    // with a service attached the context may be shared between threads
    // (qhuff_lsqpack_set_context): every call goes through svc_call, which
    // serialises the ones too large for a slot on the context's host path
    // (host_batch shares the context's staging buffers, streams and events)
    if (c && c->svc)
        return svc_call(c->svc, true, in, in_off, n, mode, out, out_off, nullptr);
    return host_batch(c, true, in, in_off, n, mode, out, out_off, nullptr);
}

extern "C" int
qhuff_decode_batch_host(qhuff_ctx *c, const uint8_t *in,
                        const uint32_t *in_off, uint32_t n, uint8_t *out,
                        uint32_t *out_off, uint8_t *status)
{
    if (c && c->svc)                      // (see qhuff_encode_batch_host)
        return svc_call(c->svc, false, in, in_off, n, 0, out, out_off, status);
    return host_batch(c, false, in, in_off, n, 0, out, out_off, status);
}

// ---- one batch over several contexts ---------------
//
// The path shards trivially -- a string's output depends on its own bytes
// and the static table only (lsqpack.c:5085-5195, 5234-5466) -- so a batch
// is cut by input bytes (qhuff_shard_cuts) into one contiguous shard per
// context, every shard runs on its own host thread (the caller's thread
// takes shard 0), and the outputs are stitched by adding each shard's base
// (the exclusive scan of the shard totals) to its offsets.  No collective:
// the only cross-shard dependency is that base.

// contexts distinct and non-null
static bool
ctxs_ok(qhuff_ctx *const *ctxs, uint32_t g)
{
    if (!ctxs || g == 0 || g > 1024)
        return false;
    for (uint32_t k = 0; k < g; ++k)
    {
        if (!ctxs[k])
            return false;
        for (uint32_t j = 0; j < k; ++j)
            if (ctxs[j] == ctxs[k])
                return false;
    }
    return true;
}

// run f(k) for k in [0, g): threads for k >= 1, the caller for k = 0;
// the first failing return code (in shard order), or QHUFF_OK
// (A shard whose thread cannot be created runs on the caller's thread after
// shard 0, in shard order: a shard only ever waits for earlier ones.)
template <class F>
static int
run_shards(uint32_t g, F f)
{
    std::vector<int> rc(g, QHUFF_OK);
    std::vector<std::thread> th;
    std::vector<uint32_t> inline_k;
    th.reserve(g ? g - 1 : 0);
    for (uint32_t k = 1; k < g; ++k)
    {
        try
        {
            th.emplace_back([&rc, &f, k] { rc[k] = f(k); });
        }
        catch (...)
        {
            inline_k.push_back(k);
        }
    }
    rc[0] = f(0);
    for (uint32_t k : inline_k)
        rc[k] = f(k);
    for (auto &t : th)
        t.join();
    for (uint32_t k = 0; k < g; ++k)
        if (rc[k])
            return rc[k];
    return QHUFF_OK;
}

static int
host_multi(qhuff_ctx *const *ctxs, uint32_t g, bool enc, const uint8_t *in,
           const uint32_t *in_off, uint32_t n, unsigned mode, uint8_t *out,
           uint32_t *out_off, uint8_t *status)
{
    if (!ctxs_ok(ctxs, g) || !in_off || !out_off || (n && (!in || !out))
            || (!enc && n && !status))
        return QHUFF_EINVAL;
    if (enc && mode != 0 && mode != 3 && mode != 5 && mode != 7)
        return QHUFF_EINVAL;
    const uint64_t bytes = (uint64_t) in_off[n] - in_off[0];
    if ((enc ? qhuff_encode_bound(bytes, n, mode) : qhuff_decode_bound(bytes, n))
            > 0xffffffffull)
        return QHUFF_ERANGE;
    std::vector<uint32_t> cuts(g + 1);
    int rc = qhuff_shard_cuts(in_off, n, g, cuts.data());
    if (rc)
        return rc;
    ShardSync sync(g);
    return run_shards(g, [&](uint32_t k) -> int {
        const uint32_t s0 = cuts[k], m = cuts[k + 1] - s0;
        const int r = host_batch(ctxs[k], enc, in, in_off + s0, m, mode, out,
                                 out_off + s0, status ? status + s0 : nullptr,
                                 &sync, k, k + 1 == g);
        if (r)
            sync.fail();
        return r;
    });
}

extern "C" int
qhuff_encode_batch_host_multi(qhuff_ctx *const *ctxs, uint32_t g,
                              const uint8_t *in, const uint32_t *in_off,
                              uint32_t n, unsigned mode, uint8_t *out,
                              uint32_t *out_off)
{
    return host_multi(ctxs, g, true, in, in_off, n, mode, out, out_off,
                      nullptr);
}

extern "C" int
qhuff_decode_batch_host_multi(qhuff_ctx *const *ctxs, uint32_t g,
                              const uint8_t *in, const uint32_t *in_off,
                              uint32_t n, uint8_t *out, uint32_t *out_off,
                              uint8_t *status)
{
    return host_multi(ctxs, g, false, in, in_off, n, 0, out, out_off, status);
}

// Device-resident shards: shard k is already on ctxs[k]'s device.  Each
// thread launches its shard and reads its total; the bases are the
// exclusive scan; with rebase, a small kernel adds shard k's base to its
// out_off on its own device (out_off then holds offsets into the
// concatenation of the shards' outputs).  Synchronous.
static int
dev_multi(qhuff_ctx *const *ctxs, uint32_t g, bool enc,
          const struct qhuff_shard *sh, unsigned mode, uint64_t *base,
          int rebase)
{
    if (!ctxs_ok(ctxs, g) || !sh || !base)
        return QHUFF_EINVAL;
    ShardSync sync(g);
    std::vector<uint64_t> bases(g + 1, 0);
    const int rc = run_shards(g, [&](uint32_t k) -> int {
        qhuff_ctx *c = ctxs[k];
        const qhuff_shard &s = sh[k];
        hipStream_t st = (hipStream_t) s.stream;
        int r = enc ? qhuff_encode_batch(c, s.in, s.in_off, s.n, mode, s.out,
                                         s.out_off, s.stream)
                    : qhuff_decode_batch(c, s.in, s.in_off, s.n, s.out,
                                         s.out_off, s.status, s.stream);
        uint32_t t = 0;
        if (!r)
        {
            hipError_t e = hipMemcpyAsync(&t, s.out_off + s.n, 4,
                                          hipMemcpyDeviceToHost, st);
            if (e == hipSuccess)
                e = hipStreamSynchronize(st);
            if (e != hipSuccess)
                r = fail(c, e, "shard total");
        }
        if (!r && c->err_host[0])
            r = mirror_error(c);
        if (r)
        {
            sync.fail();
            return r;
        }
        sync.publish(k, t);
        const uint64_t b = sync.base_of(k);
        if (b == ~0ull)
            return QHUFF_EDEVICE;
        bases[k] = b;
        if (b + t > 0xffffffffull)
            return QHUFF_ERANGE;
        if (rebase && b)
        {
            HIPCHK(c, hipSetDevice(c->device));
            HIPCHK(c, launch_rebase(s.out_off, (uint64_t) s.n + 1,
                                    (uint32_t) b, st));
            HIPCHK(c, hipStreamSynchronize(st));
        }
        if (k + 1 == g)
            bases[g] = b + t;
        return QHUFF_OK;
    });
    if (rc)
        return rc;
    memcpy(base, bases.data(), 8ull * (g + 1));
    return QHUFF_OK;
}

extern "C" int
qhuff_encode_batch_multi(qhuff_ctx *const *ctxs, uint32_t g,
                         const struct qhuff_shard *shards, unsigned mode,
                         uint64_t *base, int rebase)
{
    if (mode != 0 && mode != 3 && mode != 5 && mode != 7)
        return QHUFF_EINVAL;
    return dev_multi(ctxs, g, true, shards, mode, base, rebase);
}

extern "C" int
qhuff_decode_batch_multi(qhuff_ctx *const *ctxs, uint32_t g,
                         const struct qhuff_shard *shards, uint64_t *base,
                         int rebase)
{
    return dev_multi(ctxs, g, false, shards, 0, base, rebase);
}

// ---- low-latency service (qhuff_service.hip) -----------------------------------
//
// The resident kernel's request slots live in pinned, device-mapped host
// memory (fine-grained: the device's loads and stores of a slot go over PCIe
// and are coherent with the host's).  A call takes a free slot, writes the
// rebased offsets, the bytes and the header, then the request sequence
// number (release); it spins on the slot's done word (acquire), copies the
// results out and frees the slot.  The kernel is (re)started on demand: at
// the first call, and by a waiting call that finds the service stream idle
// (the waves leave after idle_us without requests).

struct qhuff_svc
{
    qhuff_ctx *ctx;
    hipStream_t stream;              // the resident kernel's own stream
    uint8_t *slots_h, *slots_d;      // pinned slots, host / device views
    uint32_t *ctl_h, *ctl_d;         // pinned control word: [0] stop
    uint8_t *scratch;                // device: kSvcScratchBytes per slot
    uint64_t *active;                // device: last serve time (100 MHz)
    uint32_t n_slots, grid;
    uint64_t idle_ticks, life_ticks;
    std::atomic<uint32_t> *busy;     // per slot: 0 free, 1 taken
    uint32_t *seq;                   // per slot: last posted sequence
    std::atomic<uint32_t> next_slot{0};
    std::mutex launch_mu;            // (re)launch of the kernel
    std::mutex fallback_mu;          // large requests: the context's host path
    std::atomic<uint64_t> served{0}, launches{0}, fallbacks{0};
    // steady-clock ns of the last answered request: within idle_us / 2 of
    // it the kernel cannot have left for idle, and a call skips the stream
    // query (a lock in the HIP runtime every caller would queue on)
    std::atomic<int64_t> last_done_ns{0};
    int64_t fresh_ns;
};

static inline int64_t
steady_ns()
{
    return std::chrono::duration_cast<std::chrono::nanoseconds>(
               std::chrono::steady_clock::now().time_since_epoch())
        .count();
}

static inline SvcHdr *
svc_hdr(qhuff_svc *v, uint32_t k)
{
    return (SvcHdr *) (v->slots_h + (size_t) k * kSvcSlotBytes);
}

static bool
svc_fits(const uint32_t *in_off, uint32_t n)
{
    return n <= kSvcMaxStrings && (uint64_t) in_off[n] - in_off[0] <= kSvcInCap
           && in_off[n] >= in_off[0];
}

// start the kernel if its stream is idle (a previous instance has left)
static int
svc_ensure_running(qhuff_svc *v)
{
    std::lock_guard<std::mutex> g(v->launch_mu);
    qhuff_ctx *c = v->ctx;
    const hipError_t q = hipStreamQuery(v->stream);
    if (q == hipErrorNotReady)
        return QHUFF_OK;
    if (q != hipSuccess)
        return fail(c, q, "hipStreamQuery(service)");
    HIPCHK(c, hipSetDevice(c->device));
    __atomic_store_n(&v->ctl_h[0], 0u, __ATOMIC_RELEASE);
    HIPCHK(c, hipMemsetAsync(v->active, 0, sizeof(uint64_t), v->stream));
    SvcArgs a;
    a.slots = v->slots_d;
    a.scratch = v->scratch;
    a.ctl = v->ctl_d;
    a.active = v->active;
    a.win = c->tab->win;
    a.sorted = c->tab->sorted;
    a.long2 = c->tab->long2;
    a.enc = c->tab->enc;
    a.idle_ticks = v->idle_ticks;
    a.life_ticks = v->life_ticks;
    HIPCHK(c, launch_service(a, v->grid, v->stream));
    v->launches.fetch_add(1, std::memory_order_relaxed);
    return QHUFF_OK;
}

extern "C" int
qhuff_svc_open(qhuff_ctx *c, unsigned slots, unsigned idle_us, qhuff_svc **out)
{
    if (!c || !out)
        return QHUFF_EINVAL;
    *out = nullptr;
    if (c->svc)
        return QHUFF_EINVAL;                     // one service per context
    HIPCHK(c, hipSetDevice(c->device));
    const uint32_t wpb = (uint32_t) service_waves_per_block();
    uint32_t grid = slots ? (slots + wpb - 1) / wpb : 1;
    if (grid > (uint32_t) c->n_cu / 4)
        grid = (uint32_t) c->n_cu / 4;           // at most a quarter of the CUs
    if (grid < 1)
        grid = 1;
    qhuff_svc *v = new (std::nothrow) qhuff_svc();
    if (!v)
        return QHUFF_ENOMEM;
    v->ctx = c;
    v->grid = grid;
    v->n_slots = grid * wpb;
    v->idle_ticks = 100ull * (idle_us ? idle_us : 20000u);   // 100 MHz clock
    v->fresh_ns = 500ll * (idle_us ? idle_us : 20000u);      // idle_us / 2
    v->life_ticks = 100ull * 1000000ull * 10;                // 10 s
    v->busy = new std::atomic<uint32_t>[v->n_slots];
    v->seq = new uint32_t[v->n_slots];
    for (uint32_t k = 0; k < v->n_slots; ++k)
    {
        v->busy[k].store(0);
        v->seq[k] = 0;
    }
    const size_t sb = (size_t) v->n_slots * kSvcSlotBytes;
    hipError_t e = hipHostMalloc((void **) &v->slots_h, sb,
                                 hipHostMallocMapped | hipHostMallocCoherent);
    if (e == hipSuccess)
    {
        memset(v->slots_h, 0, sb);
        e = hipHostGetDevicePointer((void **) &v->slots_d, v->slots_h, 0);
    }
    if (e == hipSuccess)
        e = hipHostMalloc((void **) &v->ctl_h, 64,
                          hipHostMallocMapped | hipHostMallocCoherent);
    if (e == hipSuccess)
    {
        memset(v->ctl_h, 0, 64);
        e = hipHostGetDevicePointer((void **) &v->ctl_d, v->ctl_h, 0);
    }
    if (e == hipSuccess)
        e = hipMalloc((void **) &v->scratch, (size_t) v->n_slots * kSvcScratchBytes);
    if (e == hipSuccess)
        e = hipMalloc((void **) &v->active, 64);
    if (e == hipSuccess)
        e = hipStreamCreateWithFlags(&v->stream, hipStreamNonBlocking);
    if (e != hipSuccess)
    {
        const int rc = fail(c, e, "service setup");
        c->svc = v;
        qhuff_svc_close(v);
        return rc;
    }
    c->svc = v;
    const int rc = svc_ensure_running(v);
    if (rc)
    {
        qhuff_svc_close(v);
        return rc;
    }
    *out = v;
    return QHUFF_OK;
}

extern "C" void
qhuff_svc_close(qhuff_svc *v)
{
    if (!v)
        return;
    qhuff_ctx *c = v->ctx;
    (void) hipSetDevice(c->device);
    if (v->ctl_h)
        __atomic_store_n(&v->ctl_h[0], 1u, __ATOMIC_RELEASE);
    if (v->stream)
    {
        (void) hipStreamSynchronize(v->stream);
        (void) hipStreamDestroy(v->stream);
    }
    if (v->scratch)
        (void) hipFree(v->scratch);
    if (v->active)
        (void) hipFree(v->active);
    if (v->slots_h)
        (void) hipHostFree(v->slots_h);
    if (v->ctl_h)
        (void) hipHostFree(v->ctl_h);
    delete[] v->busy;
    delete[] v->seq;
    if (c->svc == v)
        c->svc = nullptr;
    delete v;
}

// (qhuff_shim.cpp) whether ctx has the low-latency service attached
bool
qhuff::ctx_has_service(const qhuff_ctx *c)
{
    return c && c->svc;
}

// (qhuff_shim.cpp) one host-memory decode call whose rejected strings keep,
// as their output, the bytes decoded before the error (the DecPolicyT Keep
// kernel): the per-string entry points replay from them where the
// reference's decoder stops on an invalid string.  Through the context's
// host path, under the service's fallback lock when one is attached (the
// context may then be shared between threads).
int
qhuff::decode_keep_rejected(qhuff_ctx *c, const uint8_t *in,
                            const uint32_t *in_off, uint32_t n, uint8_t *out,
                            uint32_t *out_off, uint8_t *status)
{
    if (!c)
        return QHUFF_EINVAL;
    std::unique_lock<std::mutex> lk;
    if (c->svc)
        lk = std::unique_lock<std::mutex>(c->svc->fallback_mu);
    c->keep_rejected = true;
    const int rc = host_batch(c, false, in, in_off, n, 0, out, out_off, status);
    c->keep_rejected = false;
    return rc;
}

extern "C" int
qhuff_svc_stats(qhuff_svc *v, uint64_t *served, uint64_t *launches,
                uint64_t *fallbacks)
{
    if (!v)
        return QHUFF_EINVAL;
    if (served)
        *served = v->served.load();
    if (launches)
        *launches = v->launches.load();
    if (fallbacks)
        *fallbacks = v->fallbacks.load();
    return QHUFF_OK;
}

// Slot states (qhuff_svc::busy): free, taken by a call, or orphaned -- its
// request was posted but the call gave up on it (an error while waiting);
// an orphaned slot is free again once its done word shows that request.
constexpr uint32_t kSlotFree = 0, kSlotTaken = 1, kSlotOrphan = 2;

// take a free slot (spinning / yielding while none is); try_only: return
// n_slots at once if none is free.  A blocking take gives up after 10 s
// (every slot held by calls that never finish, e.g. a service that cannot
// run): it returns n_slots then too, and the caller reports QHUFF_EDEVICE.
static uint32_t
svc_take(qhuff_svc *v, bool try_only)
{
    uint32_t k = v->next_slot.fetch_add(1, std::memory_order_relaxed) % v->n_slots;
    const auto t0 = std::chrono::steady_clock::now();
    for (uint32_t tries = 0;; ++tries)
    {
        uint32_t z = kSlotFree;
        if (v->busy[k].compare_exchange_strong(z, kSlotTaken,
                                               std::memory_order_acquire))
            return k;
        if (z == kSlotOrphan
            && __atomic_load_n(&svc_hdr(v, k)->done, __ATOMIC_ACQUIRE) == v->seq[k]
            && v->busy[k].compare_exchange_strong(z, kSlotTaken,
                                                  std::memory_order_acquire))
            return k;                            // its abandoned request is done
        k = (k + 1) % v->n_slots;
        if (tries % v->n_slots == v->n_slots - 1)
        {
            if (try_only)
                return v->n_slots;
            if (std::chrono::steady_clock::now() - t0 > std::chrono::seconds(10))
                return v->n_slots;
            std::this_thread::yield();
        }
    }
}

// a call that stops waiting for slot k's request sq: free the slot if the
// request is done, else leave it orphaned (svc_take frees it once it is)
static void
svc_abandon(qhuff_svc *v, uint32_t k, uint32_t sq)
{
    const bool done = __atomic_load_n(&svc_hdr(v, k)->done, __ATOMIC_ACQUIRE) == sq;
    v->busy[k].store(done ? kSlotFree : kSlotOrphan, std::memory_order_release);
}

// write strings [s0, s1) of the call into slot k and post it; returns the
// request's sequence number
static uint32_t
svc_post(qhuff_svc *v, uint32_t k, bool enc, const uint8_t *in,
         const uint32_t *in_off, uint32_t s0, uint32_t s1, unsigned mode)
{
    uint8_t *sb = v->slots_h + (size_t) k * kSvcSlotBytes;
    SvcHdr *h = svc_hdr(v, k);
    const uint32_t n = s1 - s0, a0 = in_off[s0], nb = in_off[s1] - a0;
    uint32_t *so = (uint32_t *) (sb + kSvcInOffAt);
    for (uint32_t i = 0; i <= n; ++i)
        so[i] = in_off[s0 + i] - a0;
    if (nb)
        memcpy(sb + kSvcInAt, in + a0, nb);
    h->n = n;
    h->in_bytes = nb;
    h->opmode = (enc ? kSvcOpEncode : kSvcOpDecode) | (mode << 8);
    const uint32_t sq = v->seq[k] + 1 ? v->seq[k] + 1 : 1;
    v->seq[k] = sq;
    __atomic_store_n(&h->req, sq, __ATOMIC_RELEASE);
    return sq;
}

// Wait for slot k's request sq: spin on the done word; every ~50 us check
// that the kernel still runs (its waves leave after idle_us with no request
// served, and one may have left just as this request was posted); give up
// after 10 s (the slot then stays taken).
static int
svc_wait(qhuff_svc *v, uint32_t k, uint32_t sq)
{
    SvcHdr *h = svc_hdr(v, k);
    const auto t0 = std::chrono::steady_clock::now();
    auto t_chk = t0;
    for (uint32_t it = 0;; ++it)
    {
        if (__atomic_load_n(&h->done, __ATOMIC_ACQUIRE) == sq)
            return QHUFF_OK;
        if ((it & 255) == 255)
        {
            const auto now = std::chrono::steady_clock::now();
            if (now - t_chk > std::chrono::microseconds(50))
            {
                t_chk = now;
                int rc = svc_ensure_running(v);
                if (rc)
                    return rc;
                if (now - t0 > std::chrono::seconds(10))
                {
                    snprintf(v->ctx->err_msg, sizeof(v->ctx->err_msg),
                             "service request timed out");
                    return QHUFF_EDEVICE;
                }
            }
        }
        __builtin_ia32_pause();
    }
}

// slot k's result for n strings -> out + base, out_off / status (the
// piece's first string); returns its output bytes
static uint32_t
svc_collect(qhuff_svc *v, uint32_t k, bool enc, uint32_t n, uint32_t base,
            uint8_t *out, uint32_t *out_off, uint8_t *status)
{
    const uint8_t *sb = v->slots_h + (size_t) k * kSvcSlotBytes;
    const uint32_t *oo = (const uint32_t *) (sb + kSvcOutOffAt);
    const uint32_t total = oo[n];
    for (uint32_t i = 0; i < n; ++i)
        out_off[i] = base + oo[i];
    if (total)
        memcpy(out + base, sb + kSvcOutAt, total);
    if (!enc)
        memcpy(status, sb + kSvcStatusAt, n);
    return total;
}

// A call is cut into pieces of at most one staged tile each (64 strings,
// kSvcTileBytes input bytes; a longer string alone), one slot per piece: the
// service codes a one-tile piece straight from its slot, and the pieces of
// a call run on as many waves at once as there are free slots.
static int
svc_call(qhuff_svc *v, bool enc, const uint8_t *in, const uint32_t *in_off,
         uint32_t n, unsigned mode, uint8_t *out, uint32_t *out_off,
         uint8_t *status)
{
    qhuff_ctx *c = v->ctx;
    if (!in_off || !out_off || (n && (!in || !out)) || (!enc && n && !status))
        return QHUFF_EINVAL;
    if (enc && mode != 0 && mode != 3 && mode != 5 && mode != 7)
        return QHUFF_EINVAL;
    if (n == 0)
    {
        out_off[0] = 0;
        return QHUFF_OK;
    }
    for (uint32_t i = 0; i < n; ++i)             // the kernel trusts the slot
        if (in_off[i + 1] < in_off[i])
            return QHUFF_EINVAL;
    if (!svc_fits(in_off, n))
    {
        // too large for a slot: the context's host path (one caller at a time)
        std::lock_guard<std::mutex> g(v->fallback_mu);
        v->fallbacks.fetch_add(1, std::memory_order_relaxed);
        return host_batch(c, enc, in, in_off, n, mode, out, out_off, status);
    }
    constexpr uint32_t kMaxRound = 64;           // pieces in flight per call
    uint32_t base = 0;
    uint32_t s0 = 0;
    while (s0 < n)
    {
        // this round's pieces, each in its own slot (the first slot waited
        // for, further ones only while free)
        uint32_t slot[kMaxRound], p0[kMaxRound + 1], sq[kMaxRound];
        uint32_t np = 0;
        p0[0] = s0;
        while (s0 < n && np < kMaxRound)
        {
            uint32_t s1 = s0 + 1;
            while (s1 < n && s1 - s0 < (uint32_t) kWT
                   && in_off[s1 + 1] - in_off[s0] <= kSvcTileBytes)
                ++s1;
            const uint32_t k = svc_take(v, np > 0);
            if (k == v->n_slots)
            {
                if (np > 0)
                    break;                       // a partial round: go on
                snprintf(c->err_msg, sizeof(c->err_msg),
                         "service: no request slot freed within 10 s");
                return QHUFF_EDEVICE;
            }
            slot[np] = k;
            sq[np] = svc_post(v, k, enc, in, in_off, s0, s1, mode);
            p0[++np] = s1;
            s0 = s1;
        }
        int rc = QHUFF_OK;
        if (steady_ns() - v->last_done_ns.load(std::memory_order_relaxed)
                > v->fresh_ns)
            rc = svc_ensure_running(v);
        for (uint32_t j = 0; j < np; ++j)
        {
            if (!rc)
                rc = svc_wait(v, slot[j], sq[j]);
            if (rc)
            {
                // this piece and the rest of the round are abandoned: their
                // slots come back once their requests are done
                svc_abandon(v, slot[j], sq[j]);
                continue;
            }
            const uint32_t a = p0[j], m = p0[j + 1] - a;
            base += svc_collect(v, slot[j], enc, m, base, out, out_off + a,
                                enc ? nullptr : status + a);
            v->busy[slot[j]].store(kSlotFree, std::memory_order_release);
        }
        if (rc)
            return rc;
    }
    out_off[n] = base;
    v->served.fetch_add(1, std::memory_order_relaxed);
    v->last_done_ns.store(steady_ns(), std::memory_order_relaxed);
    return QHUFF_OK;
}

extern "C" int
qhuff_svc_encode(qhuff_svc *v, const uint8_t *in, const uint32_t *in_off,
                 uint32_t n, unsigned mode, uint8_t *out, uint32_t *out_off)
{
    if (!v)
        return QHUFF_EINVAL;
    return svc_call(v, true, in, in_off, n, mode, out, out_off, nullptr);
}

extern "C" int
qhuff_svc_decode(qhuff_svc *v, const uint8_t *in, const uint32_t *in_off,
                 uint32_t n, uint8_t *out, uint32_t *out_off, uint8_t *status)
{
    if (!v)
        return QHUFF_EINVAL;
    return svc_call(v, false, in, in_off, n, 0, out, out_off, status);
}

// ---- batched literal decode (pre-parsed spans, qhuff_frames.cpp) -----------

extern "C" uint64_t
qhuff_literals_bound(const struct qhuff_literal *lits, uint32_t n)
{
    uint64_t b = 16;
    for (uint32_t i = 0; lits && i < n; ++i)
        b += lits[i].huffman ? (uint64_t) lits[i].len * 8 / 5 : lits[i].len;
    return b;
}

// Huffman payloads gathered straight into the pinned stage (one copy), one
// decode launch for all of them, raw literals copied on the host meanwhile.
// Stage layout: [huff bytes | in_off | out bytes | out_off | status].
extern "C" int
qhuff_decode_literals_host(qhuff_ctx *c, const uint8_t *buf,
                           const struct qhuff_literal *lits, uint32_t n,
                           uint8_t *out, uint32_t *out_off, uint8_t *status)
{
    return qhuff_decode_literals_ex(c, buf, lits, n, 0, out, out_off, status);
}

// max_len > 0: the field-section limit -- a string that decodes (or is
// declared, raw) longer than LSXPACK_MAX_STRLEN is an error in the
// reference (header_out_grow_buf, lsqpack.c:3350-3351; 3682-3685,
// 3769-3772), whatever the kernel's status.
extern "C" int
qhuff_decode_literals_ex(qhuff_ctx *c, const uint8_t *buf,
                         const struct qhuff_literal *lits, uint32_t n,
                         uint32_t max_len, uint8_t *out, uint32_t *out_off,
                         uint8_t *status)
{
    if (!c || !out_off || (n && (!buf || !lits || !out || !status)))
        return QHUFF_EINVAL;
    HIPCHK(c, hipSetDevice(c->device));
    uint64_t hb = 0;
    uint32_t nh = 0;
    for (uint32_t i = 0; i < n; ++i)
        if (lits[i].huffman)
        {
            hb += lits[i].len;
            ++nh;
        }
    const uint64_t ob = qhuff_decode_bound(hb, nh);
    if (ob > 0xffffffffull || hb > 0xffffffffull)
        return QHUFF_ERANGE;
    const size_t o_off = up16(hb), o_out = o_off + up16(4ull * (nh + 1));
    const size_t o_oo = o_out + up16(ob), o_st = o_oo + up16(4ull * (nh + 1));
    const size_t total = o_st + up16(nh ? nh : 1);
    int rc = ensure_stage(c, total);
    if (rc)
        return rc;
    hipStream_t st = c->own_stream;
    uint32_t *hoff = (uint32_t *) (c->h_stage + o_off);
    {
        uint32_t k = 0, a = 0;
        for (uint32_t i = 0; i < n; ++i)
            if (lits[i].huffman)
            {
                memcpy(c->h_stage + a, buf + lits[i].pos, lits[i].len);
                hoff[k++] = a;
                a += lits[i].len;
            }
        hoff[k] = a;
    }
    if (nh)
    {
        // the variant from this batch (auto mode only: a pinned variant
        // needs neither the copy workers nor the scan)
        if (c->kernels == 0)
        {
            if (!c->pipe_ready && (rc = pipe_setup(c)))
                return rc;
            host_hint(c, false, hoff, nh);
        }
        HIPCHK(c, hipMemcpyAsync(c->d_stage, c->h_stage, o_out,
                                 hipMemcpyHostToDevice, st));
        rc = qhuff_decode_batch(c, c->d_stage, (const uint32_t *) (c->d_stage
                                + o_off), nh, c->d_stage + o_out,
                                (uint32_t *) (c->d_stage + o_oo),
                                c->d_stage + o_st, st);
        if (rc)
            return rc;
        if (o_st + nh - o_out <= (4u << 20))
        {
            // small: the decoded bytes' bound, sizes and status in one copy
            HIPCHK(c, hipMemcpyAsync(c->h_stage + o_out, c->d_stage + o_out,
                                     o_st + nh - o_out, hipMemcpyDeviceToHost,
                                     st));
            HIPCHK(c, hipStreamSynchronize(st));
        }
        else
        {
            // sizes and status first, then exactly the decoded bytes
            HIPCHK(c, hipMemcpyAsync(c->h_stage + o_oo, c->d_stage + o_oo,
                                     4ull * (nh + 1), hipMemcpyDeviceToHost, st));
            HIPCHK(c, hipMemcpyAsync(c->h_stage + o_st, c->d_stage + o_st, nh,
                                     hipMemcpyDeviceToHost, st));
            HIPCHK(c, hipStreamSynchronize(st));
            const uint32_t dec_total = ((const uint32_t *) (c->h_stage + o_oo))[nh];
            HIPCHK(c, hipMemcpyAsync(c->h_stage + o_out, c->d_stage + o_out,
                                     dec_total, hipMemcpyDeviceToHost, st));
            HIPCHK(c, hipStreamSynchronize(st));
        }
        if ((rc = mirror_error(c)))
            return rc;
    }
    const uint32_t *doo = (const uint32_t *) (c->h_stage + o_oo);
    const uint8_t *dst = c->h_stage + o_st;
    uint64_t o = 0;
    uint32_t k = 0;
    // max_len (field sections): the reference decodes a field line's name
    // and value into ONE header buffer, which never grows past
    // LSXPACK_MAX_STRLEN (header_out_grow_buf, lsqpack.c:3346-3351; its
    // size is a uint16 lsxpack_strlen_t): a name decoded here (NAME literal
    // of the same instruction) or a static-table name (field_ref_name_len)
    // counts against its value.  A dynamic-table name is not known to the
    // framing: that value is checked alone.
    uint32_t name_len = 0, name_instr = 0;
    bool have_name = false;
    for (uint32_t i = 0; i < n; ++i)
    {
        out_off[i] = (uint32_t) o;
        uint32_t len = lits[i].len;
        uint8_t stv = QHUFF_DEC_OK;
        const uint8_t *src = buf + lits[i].pos;
        if (lits[i].huffman)
        {
            const uint32_t a = doo[k], b = doo[k + 1];
            stv = dst[k];
            ++k;
            len = b - a;
            src = c->h_stage + o_out + a;
        }
        uint32_t lim_used = 0;
        if (max_len && lits[i].kind == QHUFF_LIT_VALUE)
            lim_used = have_name && name_instr == lits[i].instr
                     ? name_len : field_ref_name_len(buf, lits[i]);
        have_name = false;
        if (max_len && (uint64_t) lim_used + len > max_len)
            stv = QHUFF_DEC_ERROR;
        status[i] = stv;
        if (stv != QHUFF_DEC_OK)
            continue;
        if (lits[i].kind == QHUFF_LIT_NAME)
        {
            have_name = true;
            name_len = len;
            name_instr = lits[i].instr;
        }
        memcpy(out + o, src, len);
        o += len;
    }
    out_off[n] = (uint32_t) o;
    return QHUFF_OK;
}

// ---- header hashing, host buffers ----------------------------------------------

// Stage layout: [name/value bytes | offsets (2n + 1) | name_hash | nameval_hash].
// The kernel reads the caller's offsets unchanged: `in` is passed rebased by
// -off[0].
extern "C" int
qhuff_xxh32_headers_host(qhuff_ctx *c, const uint8_t *in, const uint32_t *off,
                         uint32_t n, uint32_t seed, uint32_t *name_hash,
                         uint32_t *nameval_hash)
{
    if (!c || !off || (n && (!in || !name_hash || !nameval_hash)))
        return QHUFF_EINVAL;
    if (n > 0x7fffffffu)
        return QHUFF_ERANGE;
    if (n == 0)
        return QHUFF_OK;
    HIPCHK(c, hipSetDevice(c->device));
    const uint64_t a0 = off[0], bytes = (uint64_t) off[2ull * n] - a0;
    const size_t o_off = up16(bytes), o_h1 = o_off + up16(4ull * (2ull * n + 1));
    const size_t o_h2 = o_h1 + up16(4ull * n), total = o_h2 + up16(4ull * n);
    int rc = ensure_stage(c, total);
    if (rc)
        return rc;
    hipStream_t st = c->own_stream;
    memcpy(c->h_stage, in + a0, bytes);
    memcpy(c->h_stage + o_off, off, 4ull * (2ull * n + 1));
    HIPCHK(c, hipMemcpyAsync(c->d_stage, c->h_stage, o_h1,
                             hipMemcpyHostToDevice, st));
    rc = qhuff_xxh32_headers(c, c->d_stage - a0,
                             (const uint32_t *) (c->d_stage + o_off), n, seed,
                             (uint32_t *) (c->d_stage + o_h1),
                             (uint32_t *) (c->d_stage + o_h2), st);
    if (rc)
        return rc;
    HIPCHK(c, hipMemcpyAsync(c->h_stage + o_h1, c->d_stage + o_h1,
                             total - o_h1, hipMemcpyDeviceToHost, st));
    HIPCHK(c, hipStreamSynchronize(st));
    memcpy(name_hash, c->h_stage + o_h1, 4ull * n);
    memcpy(nameval_hash, c->h_stage + o_h2, 4ull * n);
    return QHUFF_OK;
}

// ---- per-string mirrors -----------------------------------------------------

extern "C" int
qhuff_enc_enc_str(qhuff_ctx *c, unsigned prefix_bits, unsigned char *dst,
                  size_t dst_len, const unsigned char *str, unsigned str_len)
{
    if (!c || !dst || (!str && str_len) || (prefix_bits != 3
            && prefix_bits != 5 && prefix_bits != 7))
        return -1;
    uint32_t off[2] = {0, str_len};
    uint64_t bound = qhuff_encode_bound(str_len, 1, prefix_bits);
    unsigned char *tmp = (unsigned char *) malloc(bound);
    unsigned char dummy = 0;
    uint32_t oo[2];
    if (!tmp)
        return -1;
    int rc = qhuff_encode_batch_host(c, str_len ? str : &dummy, off, 1,
                                     prefix_bits, tmp, oo);
    int r = -1;
    if (rc == QHUFF_OK && oo[1] <= dst_len)
    {
        // keep dst[0] bits above the H bit (lsqpack.c:852, 863)
        unsigned char keep = dst[0] & (unsigned char) ~((1u << (prefix_bits + 1)) - 1);
        memcpy(dst, tmp, oo[1]);
        dst[0] |= keep;
        r = (int) oo[1];
    }
    free(tmp);
    return r;
}

extern "C" unsigned
qhuff_enc_str_size(qhuff_ctx *c, const unsigned char *str, unsigned str_len)
{
    if (!c || (!str && str_len))
        return 0;
    uint32_t off[2] = {0, str_len};
    uint64_t bound = qhuff_encode_bound(str_len, 1, 0);
    unsigned char *tmp = (unsigned char *) malloc(bound);
    unsigned char dummy = 0;
    uint32_t oo[2] = {0, 0};
    if (!tmp)
        return 0;
    int rc = qhuff_encode_batch_host(c, str_len ? str : &dummy, off, 1, 0, tmp,
                                     oo);
    free(tmp);
    return rc == QHUFF_OK ? oo[1] : 0;
}

// qhuff_huff_decode_ex (lsqpack_huff_decode with its full signature): see
// qhuff_shim.cpp

// ---- host helpers --------------------------------------------------------------

extern "C" int
qhuff_shard_cuts(const uint32_t *in_off, uint32_t n, uint32_t g,
                 uint32_t *cuts)
{
    if (!in_off || !cuts || g == 0)
        return QHUFF_EINVAL;
    const uint64_t a = in_off[0], tot = (uint64_t) in_off[n] - a;
    cuts[0] = 0;
    uint32_t i = 0;
    for (uint32_t k = 1; k < g; ++k)
    {
        uint64_t target = a + tot * k / g;
        // first string index whose start offset reaches the target
        uint32_t lo = i, hi = n;
        while (lo < hi)
        {
            uint32_t mid = lo + (hi - lo) / 2;
            if (in_off[mid] < target)
                lo = mid + 1;
            else
                hi = mid;
        }
        i = lo;
        cuts[k] = i;
    }
    cuts[g] = n;
    return QHUFF_OK;
}

extern "C" uint64_t
qhuff_synth_batch(uint64_t seed, uint32_t n, uint32_t min_len,
                  uint32_t max_len, const uint8_t *alphabet,
                  uint32_t alphabet_len, uint8_t *data, uint32_t *in_off)
{
    uint64_t x = seed ? seed : 0x9E3779B97F4A7C15ull;
    uint64_t pos = 0;
    const uint32_t span = max_len - min_len + 1;
    for (uint32_t i = 0; i < n; ++i)
    {
        in_off[i] = (uint32_t) pos;
        x ^= x << 13; x ^= x >> 7; x ^= x << 17;
        uint32_t len = min_len + (uint32_t) (x % span);
        for (uint32_t k = 0; k < len; ++k)
        {
            x ^= x << 13; x ^= x >> 7; x ^= x << 17;
            data[pos++] = alphabet[x % alphabet_len];
        }
    }
    in_off[n] = (uint32_t) pos;
    return pos;
}
