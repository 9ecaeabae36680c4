/*
 * lzf_api.cpp -- the C-ABI of liblzf_hip.so.
 *
 * Exports the drop-in pair of include/lzf.h (replacing src/lzf_c.c:98 and
 * src/lzf_d.c:55 behind the prototypes of src/lzf.h:76-78, 95-97) and the
 * batched device API of include/lzf_gpu.h.  There is no CPU codec in this
 * library: every call runs the HIP kernels.  Failures never abort (a server
 * must survive a transient HIP error): when no gfx950 device is usable or a
 * HIP call fails, lzf_compress returns 0 (the caller stores the value plain,
 * src/query.c:393), lzf_decompress returns 0 with errno EIO, and the batch
 * calls return a negative LZF_GPU_E* code (LZF_GPU_ENODEV without a device).
 *
 * Single calls are batches of one.  Each calling thread owns a context
 * (stream, device buffers, pinned staging), created lazily on the device
 * named by LZF_GPU_DEVICE (default 0); the caller's current device is
 * restored before returning, so Gibson's event loop never has to touch HIP.
 */
#include <errno.h>
#include <stdio.h>
#include <stdlib.h>
#include <string.h>

#include <mutex>
#include <string>
#include <thread>
#include <vector>

#include "lzf_internal.h"
#include "../../include/lzf.h"
#include "../../include/lzf_gpu.h"

#ifdef LZF_DIAG
hipError_t lzf_launch_compress_serial(const LzfBatch &b, hipStream_t s);
hipError_t lzf_launch_decompress_serial(const LzfBatch &b, hipStream_t s);
#endif

int lzf_lds_order_check(int dev);   /* lzf_selfcheck.hip */

namespace {

enum KernelGen { GEN_TABLE = 0, GEN_LANE = 1, GEN_WINDOW = 2, GEN_SERIAL = 3, GEN_WTAB = 4, GEN_TABLE_ONLY = 5 };

/* values of at most this many bytes take the lane generation by default
 * (stream cand + lane parse), larger ones the table generation: json4k
 * 1 M x 4 KiB 45.9 vs 48.7 ms (small class), text8k 1 M x 8 KiB 88.8 vs
 * 111.0 ms (table), mixed16k 256 K x 16 KiB 65.1 vs 71.4 ms (table), but
 * text64k 128 K x 64 KiB 127.4 vs 121.6 ms (the table's two-link records
 * save the parse more hops than its cand costs) */
constexpr uint32_t LANE_DEFAULT_MAX = 16384u;

/* LZF_GPU_KERNEL picks the kernel generation, read per launch so one process
 * can A/B them.  Unset: the measured routing of launch_compress (the lane
 * generation -- the stream cand kernel, lzf_stream.hip, and the lane parse,
 * lzf_lane.hip -- up to 16 KiB; the table generation, lzf_cand.hip, for values
 * of 16-64 KiB; window64 past 64 KiB and for small batches).
 * "lane": the lane generation wherever it applies; "table": the table
 * generation at any size it takes; "window": one wave per value (window64 /
 * tokpar64).  Diagnostic build only: "serial" (the single-lane first
 * generation) and "wtab" (the window-parse generation, lzf_wparse.hip, a
 * measured prototype that is not routed).  All are bit-exact; the GPU tests
 * cross-check them. */
KernelGen kernel_gen()
{
    const char *e = getenv("LZF_GPU_KERNEL");
#ifdef LZF_DIAG
    if (e && !strcmp(e, "serial")) return GEN_SERIAL;
    if (e && !strcmp(e, "wtab")) return GEN_WTAB;
#endif
    if (e && !strcmp(e, "window")) return GEN_WINDOW;
    if (e && !strcmp(e, "lane")) return GEN_LANE;
    if (e && !strcmp(e, "table")) return GEN_TABLE_ONLY;
    return GEN_TABLE;
}

bool device_ok(int dev)
{
    static std::mutex mu;
    static int checked[64];      /* 0 unknown, 1 ok, -1 bad */
    if (dev < 0 || dev >= 64) return false;
    std::lock_guard<std::mutex> lk(mu);
    if (!checked[dev]) {
        hipDeviceProp_t prop;
        checked[dev] = (hipGetDeviceProperties(&prop, dev) == hipSuccess &&
                        strstr(prop.gcnArchName, "gfx950") != nullptr) ? 1 : -1;
    }
    return checked[dev] == 1;
}

/* The table, lane and window generations need the LDS to run a wave's
 * same-address ds_mskor_rtn_b32 in lane order (lzf_selfcheck.hip).  Checked
 * per device before their first launch (on the probe's own stream, so the
 * caller's stream and the rest of the device are not synchronised); where it
 * does not hold, compress batches go to window64.  Only a definite answer is
 * kept: a probe that could not run (an allocation or launch failure under
 * load) routes this batch to window64 and is tried again on the next one.
 * LZF_GPU_FORCE_ORDER_FAIL=1 makes the check report a violation (tests of
 * the fallback).  A caller that captures compress launches in a HIP graph
 * runs lzf_gpu_selfcheck() first, outside the capture. */
int g_order[64];                     /* 0 unchecked, 1 held, -1 violated */
int g_order_last[64];                /* the last probe's outcome, -2: it could not run */
std::mutex g_order_mu;

int lds_order_state(bool run)
{
    int dev = 0;
    if (hipGetDevice(&dev) != hipSuccess || dev < 0 || dev >= 64) return -2;
    std::lock_guard<std::mutex> lk(g_order_mu);
    if (!g_order[dev] && run) {
        const char *f = getenv("LZF_GPU_FORCE_ORDER_FAIL");
        const int bad = (f && *f == '1') ? 1 : lzf_lds_order_check(dev);
        g_order_last[dev] = bad == 0 ? 1 : bad > 0 ? -1 : -2;
        if (bad >= 0) g_order[dev] = g_order_last[dev];
        return g_order_last[dev];
    }
    return g_order[dev] ? g_order[dev] : g_order_last[dev];
}

bool lds_order_ok() { return lds_order_state(true) == 1; }

int current_device_ok()
{
    int dev = -1;
    if (hipGetDevice(&dev) != hipSuccess) return LZF_GPU_ENODEV;
    return device_ok(dev) ? LZF_GPU_OK : LZF_GPU_ENODEV;
}

/* Compress scratch (records/cand words + inserted bitmap), ONE per device,
 * shared by every host thread under a mutex and grown on demand (cap:
 * scratch_limit).  The mutex is held while a batch is enqueued; a batch on
 * another stream than the previous user first waits for that user's
 * kernels (an event), so concurrent callers stay correct.  lzf_gpu_release()
 * frees it. */
struct Scratch {
    std::mutex mu;
    void *p = nullptr;
    size_t cap = 0;
    hipEvent_t ev = nullptr;
    hipStream_t last = nullptr;
    bool used = false;
#ifdef LZF_DIAG
    hipStream_t aux = nullptr;      /* kernel-2 stream of the chunk pipeline */
    hipEvent_t pev[4] = {nullptr, nullptr, nullptr, nullptr};
#endif
};

Scratch g_scratch[64];

/* Scratch cap: LZF_GPU_SCRATCH_MB if set, else half of the device memory
 * free when the scratch grows (at least 1 GiB): a whole BASELINE batch
 * (256 K x 64 KiB: 67 GiB of records) then runs as one chunk, and a caller
 * that holds most of the device still gets chunked, not refused. */
size_t scratch_limit(size_t held)
{
    const char *e = getenv("LZF_GPU_SCRATCH_MB");
    if (e) {
        unsigned long long mb = strtoull(e, nullptr, 10);
        if (mb < 1) mb = 1;
        return (size_t)mb << 20;
    }
    size_t fr = 0, tot = 0;
    if (hipMemGetInfo(&fr, &tot) != hipSuccess) return (size_t)40 << 30;
    size_t lim = (fr + held) / 2;
    return lim > ((size_t)1 << 30) ? lim : ((size_t)1 << 30);
}

void scratch_free(Scratch &S)
{
    if (S.p) {
        if (S.used && S.ev) (void)hipEventSynchronize(S.ev);
        (void)hipFree(S.p);
    }
    S.p = nullptr;
    S.cap = 0;
    S.used = false;
}

enum ScratchUser { SU_LANE = 0, SU_TABLE = 1, SU_WTAB = 2 };
/* chunks of this thread's last scratch-bound compress launch (kernel_info) */
thread_local uint32_t g_last_chunks = 0;

hipError_t lane_compress(const LzfBatch &b, hipStream_t s, ScratchUser who)
{
    const bool table = who == SU_TABLE;
    int dev = 0;
    hipError_t e = hipGetDevice(&dev);
    if (e != hipSuccess) return e;
    Scratch &S = g_scratch[dev & 63];
    std::lock_guard<std::mutex> lk(S.mu);
#ifdef LZF_DIAG
    const size_t per = who == SU_WTAB ? lzf_wtab_scratch_per_value(b.max_len)
                       : table        ? lzf_table_scratch_per_value(b.max_len)
                                      : lzf_lane_scratch_per_value(b.max_len);
#else
    const size_t per = table ? lzf_table_scratch_per_value(b.max_len) : lzf_lane_scratch_per_value(b.max_len);
#endif
    size_t want = per * (size_t)b.count + 512;
    const size_t lim = scratch_limit(S.cap);
    if (want > lim) want = lim;
    if (want < 2 * per + 1024) want = 2 * per + 1024;     /* two pipeline halves */
    /* an explicit cap binds even when an earlier batch grew the scratch past
     * it: the buffer is given back and re-made at the cap */
    const bool capped = getenv("LZF_GPU_SCRATCH_MB") != nullptr;
    if (capped && S.cap > want && S.cap > lim) scratch_free(S);
    if (S.cap < want) {
        scratch_free(S);
        /* short of device memory: a smaller scratch only means more chunks */
        const size_t least = 2 * per + 1024;
        while ((e = hipMalloc(&S.p, want)) != hipSuccess && want > least) {
            (void)hipGetLastError();
            want = want / 2 > least ? want / 2 : least;
        }
        if (e != hipSuccess) {
            S.p = nullptr;
            return e;
        }
        S.cap = want;
    }
    if (!S.ev && (e = hipEventCreateWithFlags(&S.ev, hipEventDisableTiming)) != hipSuccess) return e;
    if (S.used && S.last != s && (e = hipStreamWaitEvent(s, S.ev, 0)) != hipSuccess) return e;
    /* the chunk size comes from the usable scratch: the buffer, or the cap
     * when one is set below it */
    const size_t use = capped && lim < S.cap ? (lim > 2 * per + 1024 ? lim : 2 * per + 1024) : S.cap;
    if (table) {
        e = lzf_launch_compress_table(b, s, S.p, use, &g_last_chunks);
    }
#ifdef LZF_DIAG
    else if (who == SU_WTAB) {
        e = lzf_launch_compress_wtab(b, s, S.p, use, &g_last_chunks);
    }
#endif
    else {
#ifdef LZF_DIAG
        const char *ff = getenv("LZF_GPU_LANE_FORCE_FIX");
        /* LZF_GPU_LANE_PIPE=1 overlaps the two kernels of consecutive chunks
         * on two streams (both kernels hold LDS and do not co-reside well) */
        const char *pp = getenv("LZF_GPU_LANE_PIPE");
        const bool pipe = pp && *pp == '1';
        if (pipe && !S.aux) {
            if ((e = hipStreamCreateWithFlags(&S.aux, hipStreamNonBlocking)) != hipSuccess) return e;
            for (int k = 0; k < 4; k++)
                if ((e = hipEventCreateWithFlags(&S.pev[k], hipEventDisableTiming)) != hipSuccess) return e;
        }
        e = lzf_launch_compress_lane(b, s, S.p, use, (ff && *ff == '1') ? 1u : 0u, pipe ? S.aux : nullptr,
                                     pipe ? S.pev : nullptr, &g_last_chunks);
#else
        e = lzf_launch_compress_lane(b, s, S.p, use, 0u, nullptr, nullptr, &g_last_chunks);
#endif
    }
    if (e != hipSuccess) return e;
    e = hipEventRecord(S.ev, s);
    S.last = s;
    S.used = true;
    return e;
}

/* smallest batch the lane / table generations take (LZF_GPU_LANE_MIN
 * overrides): below it window64's one wave per value finishes first, since
 * the parse's time has a floor of one whole value's parse per lane.
 * tools/crossover.py, round 4, the routed generations (stream cand + lane
 * parse up to 16 KiB, table above) vs window64, compress ms
 * (profiles/r04/xo_*.txt): json 4 KiB 7.02 vs 6.61 at 96 K values, 7.71 vs
 * 8.78 at 128 K; text 8 KiB 11.21 vs 11.31 at 32 K; mixed 16 KiB 24.80 vs
 * 20.07 at 32 K, 26.37 vs 29.86 at 48 K; text 64 KiB 77.22 vs 69.47 at 24 K,
 * 80.45 vs 92.62 at 32 K. */
uint32_t lane_min_count(uint32_t max_len)
{
    const char *e = getenv("LZF_GPU_LANE_MIN");
    if (e) return (uint32_t)strtoul(e, nullptr, 10);
    if (max_len <= 4096u) return 114688u;
    if (max_len <= 8192u) return 32768u;
    if (max_len <= 16384u) return 45056u;
    return 28672u;
}

hipError_t launch_compress(const LzfBatch &b, hipStream_t s)
{
    const KernelGen g = kernel_gen();
    if (g != GEN_WINDOW && g != GEN_SERIAL && !lds_order_ok()) return lzf_launch_compress(b, s);
    switch (g) {
#ifdef LZF_DIAG
    case GEN_SERIAL: return lzf_launch_compress_serial(b, s);
#endif
    case GEN_WINDOW: return lzf_launch_compress(b, s);
    case GEN_LANE:
        return (lzf_lane_compress_supported(b.max_len) && b.count >= lane_min_count(b.max_len))
                   ? lane_compress(b, s, SU_LANE)
                   : lzf_launch_compress(b, s);
#ifdef LZF_DIAG
    case GEN_WTAB:
        return lzf_wtab_compress_supported(b.max_len) ? lane_compress(b, s, SU_WTAB) : lzf_launch_compress(b, s);
#endif
    case GEN_TABLE_ONLY:
        return (lzf_table_compress_supported(b.max_len) && b.count >= lane_min_count(b.max_len))
                   ? lane_compress(b, s, SU_TABLE)
                   : lzf_launch_compress(b, s);
    default:
        /* batches with values past 64 KiB, and small batches, go to the window
         * generation: the parse runs one value per lane, so its time has a
         * floor of one whole value's parse (~5 ms); below the crossover one
         * wave per value finishes first (tools/crossover.py).  Values of at
         * most LANE_DEFAULT_MAX bytes take the lane generation (the stream
         * cand kernel, lzf_stream.hip, and the lane parse), larger ones the
         * table generation (two-link records, lzf_cand.hip) */
        if (b.count < lane_min_count(b.max_len) || !lzf_table_compress_supported(b.max_len))
            return lzf_launch_compress(b, s);
        /* the lane generation where its kernel 1 takes the batch (a
         * diagnostic LZF_GPU_CAND=small stops at 4 KiB), else the table one */
        return lane_compress(b, s, b.max_len <= LANE_DEFAULT_MAX && lzf_lane_compress_supported(b.max_len)
                                       ? SU_LANE : SU_TABLE);
    }
}

/* The lane decoder (one lane per stream, diagnostic build) is bit-exact but,
 * streaming 64 values per wave through L2, slower than pipe / tokpar64 on
 * the BASELINE shapes; it runs only when
 * LZF_GPU_DECOMPRESS=lane asks for it. */
bool lane_decoder()
{
#ifdef LZF_DIAG
    const char *e = getenv("LZF_GPU_DECOMPRESS");
    return e && !strcmp(e, "lane");
#else
    return false;                    /* the lane decoder is in the diagnostic build only */
#endif
}

hipError_t launch_decompress(const LzfBatch &b, hipStream_t s)
{
    switch (kernel_gen()) {
#ifdef LZF_DIAG
    case GEN_SERIAL: return lzf_launch_decompress_serial(b, s);
    default: return lane_decoder() ? lzf_launch_decompress_lane(b, s) : lzf_launch_decompress(b, s);
#else
    default: return lzf_launch_decompress(b, s);
#endif
    }
}

/* Library failures inside the host-memory paths are thrown as LzfFail and
 * turned into an LZF_GPU_E* code at the C boundary (never abort: a transient
 * HIP error must not take the server down). */
struct LzfFail {
    int code;
};

int code_of(hipError_t e)
{
    if (e == hipErrorOutOfMemory || e == hipErrorMemoryAllocation) return LZF_GPU_ENOMEM;
    if (e == hipErrorNoDevice || e == hipErrorInvalidDevice) return LZF_GPU_ENODEV;
    return LZF_GPU_ELAUNCH;
}

void check(hipError_t e, const char *what)
{
    if (e == hipSuccess) return;
    static bool said = false;
    if (!said) {
        said = true;
        fprintf(stderr, "liblzf_hip: %s failed: %s\n", what, hipGetErrorString(e));
    }
    (void)hipGetLastError();
    throw LzfFail{code_of(e)};
}

struct DeviceGuard {
    int prev = -1;
    explicit DeviceGuard(int dev)
    {
        if (hipGetDevice(&prev) != hipSuccess) prev = -1;
        if (prev != dev) {
            check(hipSetDevice(dev), "hipSetDevice");
        }
    }
    ~DeviceGuard()
    {
        int cur = -1;
        if (prev >= 0 && hipGetDevice(&cur) == hipSuccess && cur != prev) (void)hipSetDevice(prev);
    }
};

/* Growable device / pinned buffers of one thread. */
struct Buf {
    void *p = nullptr;
    size_t cap = 0;
    bool pinned = false;
    void *get(size_t need)
    {
        if (need == 0) need = 1;
        if (need <= cap) return p;
        size_t want = need + need / 4 + 256;
        if (p) { pinned ? (void)hipHostFree(p) : (void)hipFree(p); }
        p = nullptr;
        cap = 0;
        hipError_t e = pinned ? hipHostMalloc(&p, want, hipHostMallocDefault) : hipMalloc(&p, want);
        if (e != hipSuccess) {
            p = nullptr;
            check(e, pinned ? "hipHostMalloc" : "hipMalloc");
        }
        cap = want;
        return p;
    }
    void release()
    {
        if (p) { pinned ? (void)hipHostFree(p) : (void)hipFree(p); }
        p = nullptr;
        cap = 0;
    }
};

struct Meta {               /* one value's descriptor, packed for one copy */
    uint64_t in_off, out_off;
    uint32_t in_len, out_cap, out_len;
    int32_t err;
};

/* One stage of the chunked host pipeline: its own stream, pinned and device
 * buffers, and the chunk it holds until the results are copied out. */
struct Slot {
    hipStream_t stream = nullptr;
    hipEvent_t done = nullptr;
    Buf d_in, d_out, d_meta;
    Buf h_in{nullptr, 0, true}, h_out{nullptr, 0, true}, h_meta{nullptr, 0, true};
    uint32_t first = 0, count = 0;
    bool busy = false;
};

struct Ctx {
    int dev = 0;
    bool ok = false;
    hipStream_t stream = nullptr;
    Buf d_in, d_out, d_meta;
    Buf h_in{nullptr, 0, true}, h_out{nullptr, 0, true}, h_meta{nullptr, 0, true};
    Slot slot[2];
    Ctx()
    {
        const char *e = getenv("LZF_GPU_DEVICE");
        dev = e ? atoi(e) : 0;
        int n = 0;
        if (hipGetDeviceCount(&n) != hipSuccess || dev < 0 || dev >= n || !device_ok(dev)) {
            fprintf(stderr, "liblzf_hip: no gfx950 device %d (devices: %d); the codec runs on the GPU only\n", dev,
                    n);
            return;
        }
        int prev = -1;
        (void)hipGetDevice(&prev);
        (void)hipSetDevice(dev);
        ok = hipStreamCreateWithFlags(&stream, hipStreamNonBlocking) == hipSuccess;
        if (prev >= 0) (void)hipSetDevice(prev);
    }
    /* the buffers of this thread (at its exit, or lzf_gpu_release) */
    void release()
    {
        if (!ok) return;
        int prev = -1;
        (void)hipGetDevice(&prev);
        (void)hipSetDevice(dev);
        if (stream) (void)hipStreamSynchronize(stream);
        for (auto &sl : slot) {
            if (sl.stream) (void)hipStreamSynchronize(sl.stream);
            for (Buf *b : {&sl.d_in, &sl.d_out, &sl.d_meta, &sl.h_in, &sl.h_out, &sl.h_meta}) b->release();
            sl.busy = false;
        }
        for (Buf *b : {&d_in, &d_out, &d_meta, &h_in, &h_out, &h_meta}) b->release();
        if (prev >= 0) (void)hipSetDevice(prev);
    }
    ~Ctx() { release(); }
};

Ctx &ctx()
{
    static thread_local Ctx c;
    if (!c.ok) throw LzfFail{LZF_GPU_ENODEV};
    return c;
}

/* Run f(lo, hi) over [0, n) split into up to `threads` ranges. */
template <class F> void parallel_ranges(uint32_t n, uint32_t threads, F f)
{
    if (threads <= 1 || n < 2u * threads) {
        f(0u, n);
        return;
    }
    std::vector<std::thread> ts;
    const uint32_t per = (n + threads - 1u) / threads;
    for (uint32_t t = 1; t < threads; t++) {
        const uint32_t lo = t * per, hi = lo + per < n ? lo + per : n;
        if (lo < hi) ts.emplace_back([=]() { f(lo, hi); });
    }
    f(0u, per < n ? per : n);
    for (auto &t : ts) t.join();
}

uint32_t host_threads()
{
    const char *e = getenv("LZF_GPU_HOST_THREADS");
    if (e) return (uint32_t)atoi(e) > 0 ? (uint32_t)atoi(e) : 1u;
    const unsigned hc = std::thread::hardware_concurrency();
    return hc >= 8u ? 8u : (hc ? hc : 1u);
}

/* Large host batches: values in chunks through two slots on two streams.
 * The CPU gathers chunk k+1's values (several threads) while chunk k moves
 * over PCIe and runs; results are scattered back once a slot comes round
 * again.  Each chunk's values are packed (inputs back to back, outputs at
 * their caps back to back), so only their bytes cross the bus. */
int host_batch_pipelined(bool compress, const uint8_t *in, const uint64_t *in_off, const uint32_t *in_len,
                         uint8_t *out, const uint64_t *out_off, const uint32_t *out_cap, uint32_t *out_len,
                         int32_t *err, uint32_t count, uint64_t chunk_in, uint64_t chunk_out)
{
    Ctx &c = ctx();
    DeviceGuard g(c.dev);
    const uint32_t threads = host_threads();
    for (auto &sl : c.slot) {
        if (!sl.stream) check(hipStreamCreateWithFlags(&sl.stream, hipStreamNonBlocking), "hipStreamCreate");
        if (!sl.done) check(hipEventCreateWithFlags(&sl.done, hipEventDisableTiming), "hipEventCreate");
        sl.busy = false;
    }
    const size_t mrec = 2 * sizeof(uint64_t) + 3 * sizeof(uint32_t) + sizeof(int32_t);
    /* results of a finished slot back to the caller's arrays */
    auto drain = [&](Slot &sl) {
        if (!sl.busy) return;
        check(hipEventSynchronize(sl.done), "hipEventSynchronize");
        const uint32_t n = sl.count;
        const uint64_t *m_out_off = (const uint64_t *)sl.h_meta.p + n;
        const uint32_t *m_out_len = (const uint32_t *)(m_out_off + n) + 2u * n;
        const int32_t *m_err = (const int32_t *)(m_out_len + n);
        const uint8_t *h_out = (const uint8_t *)sl.h_out.p;
        parallel_ranges(n, threads, [&](uint32_t lo, uint32_t hi) {
            for (uint32_t k = lo; k < hi; k++) {
                const uint32_t i = sl.first + k;
                out_len[i] = m_out_len[k];
                if (err) err[i] = m_err[k];
                if (m_out_len[k]) memcpy(out + out_off[i], h_out + m_out_off[k], m_out_len[k]);
            }
        });
        sl.busy = false;
    };
    uint32_t i0 = 0, k = 0;
    while (i0 < count) {
        /* the chunk: values [i0, i1) */
        uint64_t bin = 0, bout = 0;
        uint32_t i1 = i0, max_len = 0;
        while (i1 < count) {
            const uint64_t li = in_len[i1] ? in_len[i1] : 1u;     /* a 0-length stream reads 1 byte */
            if (i1 > i0 && (bin + li > chunk_in || bout + out_cap[i1] > chunk_out)) break;
            bin += li;
            bout += out_cap[i1];
            const uint32_t l = compress ? in_len[i1] : out_cap[i1];
            if (l > max_len) max_len = l;
            i1++;
        }
        Slot &sl = c.slot[k & 1u];
        drain(sl);
        const uint32_t n = i1 - i0;
        uint8_t *h_in = (uint8_t *)sl.h_in.get(bin);
        uint8_t *h_meta = (uint8_t *)sl.h_meta.get((size_t)n * mrec);
        uint8_t *d_in = (uint8_t *)sl.d_in.get(bin);
        uint8_t *d_out = (uint8_t *)sl.d_out.get(bout);
        uint8_t *d_meta = (uint8_t *)sl.d_meta.get((size_t)n * mrec);
        sl.h_out.get(bout);
        uint64_t *m_in_off = (uint64_t *)h_meta, *m_out_off = m_in_off + n;
        uint32_t *m_in_len = (uint32_t *)(m_out_off + n), *m_out_cap = m_in_len + n;
        {
            uint64_t a = 0, b = 0;
            for (uint32_t j = 0; j < n; j++) {
                const uint32_t i = i0 + j;
                m_in_off[j] = a;
                m_out_off[j] = b;
                m_in_len[j] = in_len[i];
                m_out_cap[j] = out_cap[i];
                a += in_len[i] ? in_len[i] : 1u;
                b += out_cap[i];
            }
        }
        parallel_ranges(n, threads, [&](uint32_t lo, uint32_t hi) {
            for (uint32_t j = lo; j < hi; j++) {
                const uint32_t i = i0 + j;
                memcpy(h_in + m_in_off[j], in + in_off[i], in_len[i] ? in_len[i] : 1u);
            }
        });
        const size_t res_off = (uint8_t *)(m_out_cap + n) - h_meta;
        check(hipMemcpyAsync(d_in, h_in, bin, hipMemcpyHostToDevice, sl.stream), "hipMemcpyAsync");
        check(hipMemcpyAsync(d_meta, h_meta, res_off, hipMemcpyHostToDevice, sl.stream), "hipMemcpyAsync");
        LzfBatch b{};
        b.in = d_in;
        b.in_off = (const uint64_t *)d_meta;
        b.out_off = b.in_off + n;
        b.in_len = (const uint32_t *)(b.out_off + n);
        b.out_cap = b.in_len + n;
        b.out_len = (uint32_t *)(b.out_cap + n);
        b.err = (int32_t *)(b.out_len + n);
        b.out = d_out;
        b.count = n;
        b.max_len = max_len;
        check(compress ? launch_compress(b, sl.stream) : launch_decompress(b, sl.stream), "kernel launch");
        check(hipMemcpyAsync(h_meta + res_off, d_meta + res_off, (size_t)n * mrec - res_off,
                             hipMemcpyDeviceToHost, sl.stream), "hipMemcpyAsync");
        check(hipMemcpyAsync(sl.h_out.p, d_out, bout, hipMemcpyDeviceToHost, sl.stream), "hipMemcpyAsync");
        check(hipEventRecord(sl.done, sl.stream), "hipEventRecord");
        sl.first = i0;
        sl.count = n;
        sl.busy = true;
        i0 = i1;
        k++;
    }
    drain(c.slot[k & 1u]);
    drain(c.slot[(k + 1u) & 1u]);
    return LZF_GPU_OK;
}

/* Host batch: stage arena + descriptors, run, copy back. */
int host_batch(bool compress, const uint8_t *in, const uint64_t *in_off, const uint32_t *in_len,
               uint8_t *out, const uint64_t *out_off, const uint32_t *out_cap, uint32_t *out_len,
               int32_t *err, uint32_t count)
{
    if (!count || !in || !in_off || !in_len || !out || !out_off || !out_cap || !out_len)
        return LZF_GPU_EARG;
    {
        /* large batches whose outputs are not much bigger than their inputs
         * (compress, or decompress with caps near the values' sizes) go
         * through the chunked pipeline */
        uint64_t sin = 0, sout = 0;
        for (uint32_t i = 0; i < count; i++) {
            sin += in_len[i] ? in_len[i] : 1u;
            sout += out_cap[i];
        }
        const uint64_t chunk = 32ull << 20;
        if (sin >= 2 * chunk && sout <= 4 * sin)
            return host_batch_pipelined(compress, in, in_off, in_len, out, out_off, out_cap, out_len, err,
                                        count, chunk, 4 * chunk);
    }
    Ctx &c = ctx();
    DeviceGuard g(c.dev);
    uint64_t in_end = 0, out_end = 0;
    uint32_t max_len = 0;
    for (uint32_t i = 0; i < count; i++) {
        uint64_t ie = in_off[i] + (in_len[i] ? in_len[i] : 1u);   /* a 0-length stream reads 1 byte */
        uint64_t oe = out_off[i] + out_cap[i];
        if (ie > in_end) in_end = ie;
        if (oe > out_end) out_end = oe;
        uint32_t l = compress ? in_len[i] : out_cap[i];
        if (l > max_len) max_len = l;
    }
    size_t meta_bytes = (size_t)count * (2 * sizeof(uint64_t) + 3 * sizeof(uint32_t) + sizeof(int32_t));
    uint8_t *h_in = (uint8_t *)c.h_in.get(in_end);
    uint8_t *h_meta = (uint8_t *)c.h_meta.get(meta_bytes);
    uint8_t *d_in = (uint8_t *)c.d_in.get(in_end);
    uint8_t *d_out = (uint8_t *)c.d_out.get(out_end);
    uint8_t *d_meta = (uint8_t *)c.d_meta.get(meta_bytes);
    memcpy(h_in, in, in_end);
    uint64_t *m_in_off = (uint64_t *)h_meta;
    uint64_t *m_out_off = m_in_off + count;
    uint32_t *m_in_len = (uint32_t *)(m_out_off + count);
    uint32_t *m_out_cap = m_in_len + count;
    uint32_t *m_out_len = m_out_cap + count;
    int32_t *m_err = (int32_t *)(m_out_len + count);
    memcpy(m_in_off, in_off, count * sizeof(uint64_t));
    memcpy(m_out_off, out_off, count * sizeof(uint64_t));
    memcpy(m_in_len, in_len, count * sizeof(uint32_t));
    memcpy(m_out_cap, out_cap, count * sizeof(uint32_t));
    size_t res_off = (uint8_t *)m_out_len - h_meta;
    check(hipMemcpyAsync(d_in, h_in, in_end, hipMemcpyHostToDevice, c.stream), "hipMemcpyAsync");
    check(hipMemcpyAsync(d_meta, h_meta, res_off, hipMemcpyHostToDevice, c.stream), "hipMemcpyAsync");
    LzfBatch b{};
    b.in = d_in;
    b.in_off = (const uint64_t *)d_meta;
    b.out_off = b.in_off + count;
    b.in_len = (const uint32_t *)(b.out_off + count);
    b.out_cap = b.in_len + count;
    b.out_len = (uint32_t *)(b.out_cap + count);
    b.err = (int32_t *)(b.out_len + count);
    b.out = d_out;
    b.count = count;
    b.max_len = max_len;
    check(compress ? launch_compress(b, c.stream) : launch_decompress(b, c.stream), "kernel launch");
    check(hipMemcpyAsync(h_meta + res_off, d_meta + res_off, meta_bytes - res_off,
                         hipMemcpyDeviceToHost, c.stream), "hipMemcpyAsync");
    check(hipStreamSynchronize(c.stream), "hipStreamSynchronize");
    memcpy(out_len, m_out_len, count * sizeof(uint32_t));
    if (err) memcpy(err, m_err, count * sizeof(int32_t));
    /* copy back only the produced bytes of each value */
    uint64_t lo = ~0ull, hi = 0;
    for (uint32_t i = 0; i < count; i++) {
        if (!m_out_len[i]) continue;
        if (out_off[i] < lo) lo = out_off[i];
        if (out_off[i] + m_out_len[i] > hi) hi = out_off[i] + m_out_len[i];
    }
    if (hi > lo) {
        uint8_t *h_out = (uint8_t *)c.h_out.get(hi - lo);
        check(hipMemcpyAsync(h_out, d_out + lo, hi - lo, hipMemcpyDeviceToHost, c.stream),
              "hipMemcpyAsync");
        check(hipStreamSynchronize(c.stream), "hipStreamSynchronize");
        for (uint32_t i = 0; i < count; i++)
            if (m_out_len[i]) memcpy(out + out_off[i], h_out + (out_off[i] - lo), m_out_len[i]);
    }
    return LZF_GPU_OK;
}

/* host_batch with the failure of a library call as a return code; the
 * streams of the thread's context are drained so its buffers are free */
int host_batch_rc(bool compress, const uint8_t *in, const uint64_t *in_off, const uint32_t *in_len,
                  uint8_t *out, const uint64_t *out_off, const uint32_t *out_cap, uint32_t *out_len,
                  int32_t *err, uint32_t count)
{
    try {
        return host_batch(compress, in, in_off, in_len, out, out_off, out_cap, out_len, err, count);
    } catch (const LzfFail &f) {
        try {
            Ctx &c = ctx();
            if (c.stream) (void)hipStreamSynchronize(c.stream);
            for (auto &sl : c.slot) {
                if (sl.stream) (void)hipStreamSynchronize(sl.stream);
                sl.busy = false;
            }
            (void)hipGetLastError();
        } catch (const LzfFail &) {
        }
        return f.code;
    }
}

/* decoded sizes of host streams (the pre-pass of lzf_dsize.hip) */
int host_dsize(const uint8_t *in, const uint64_t *in_off, const uint32_t *in_len, uint32_t *out_size,
               int32_t *err, uint32_t count, uint32_t limit)
{
    if (!count || !in || !in_off || !in_len || !out_size || !err) return LZF_GPU_EARG;
    try {
        Ctx &c = ctx();
        DeviceGuard g(c.dev);
        uint64_t in_end = 0;
        for (uint32_t i = 0; i < count; i++) {
            const uint64_t ie = in_off[i] + (in_len[i] ? in_len[i] : 1u);   /* a 0-length stream reads 1 byte */
            if (ie > in_end) in_end = ie;
        }
        const size_t mb = (size_t)count * (sizeof(uint64_t) + 3 * sizeof(uint32_t));
        uint8_t *h_in = (uint8_t *)c.h_in.get(in_end), *h_meta = (uint8_t *)c.h_meta.get(mb);
        uint8_t *d_in = (uint8_t *)c.d_in.get(in_end), *d_meta = (uint8_t *)c.d_meta.get(mb);
        memcpy(h_in, in, in_end);
        memcpy(h_meta, in_off, count * sizeof(uint64_t));
        memcpy(h_meta + count * sizeof(uint64_t), in_len, count * sizeof(uint32_t));
        const size_t res = count * (sizeof(uint64_t) + sizeof(uint32_t));
        check(hipMemcpyAsync(d_in, h_in, in_end, hipMemcpyHostToDevice, c.stream), "hipMemcpyAsync");
        check(hipMemcpyAsync(d_meta, h_meta, res, hipMemcpyHostToDevice, c.stream), "hipMemcpyAsync");
        check(lzf_launch_dsize(d_in, (const uint64_t *)d_meta, (const uint32_t *)(d_meta + count * sizeof(uint64_t)),
                               (uint32_t *)(d_meta + res), (int32_t *)(d_meta + res + count * sizeof(uint32_t)), count,
                               limit, c.stream),
              "kernel launch");
        check(hipMemcpyAsync(h_meta + res, d_meta + res, mb - res, hipMemcpyDeviceToHost, c.stream),
              "hipMemcpyAsync");
        check(hipStreamSynchronize(c.stream), "hipStreamSynchronize");
        memcpy(out_size, h_meta + res, count * sizeof(uint32_t));
        memcpy(err, h_meta + res + count * sizeof(uint32_t), count * sizeof(int32_t));
        return LZF_GPU_OK;
    } catch (const LzfFail &f) {
        return f.code;
    }
}

}  // namespace

extern "C" {

/* Single calls are batches of one.  A failure of the device path (no usable
 * gfx950, a HIP error) is reported, never aborted on: lzf_compress returns 0,
 * which the caller already reads as "store the value plain"
 * (src/query.c:393-397); lzf_decompress returns 0 with errno EIO, an errno the
 * reference codec never sets (src/lzf.h:85-91 lists E2BIG and EINVAL). */
unsigned int lzf_compress(const void *const in_data, unsigned int in_len, void *out_data,
                          unsigned int out_len)
{
    if (!in_len || !out_len) return 0;                    /* src/lzf_c.c:131 */
    if (!in_data || !out_data) return 0;
    uint64_t zero = 0;
    uint32_t res = 0;
    const int rc = host_batch_rc(true, (const uint8_t *)in_data, &zero, &in_len, (uint8_t *)out_data, &zero,
                                 &out_len, &res, nullptr, 1);
    return rc == LZF_GPU_OK ? res : 0u;
}

unsigned int lzf_decompress(const void *const in_data, unsigned int in_len, void *out_data,
                            unsigned int out_len)
{
    uint8_t none = 0;
    if (!in_data || (!out_data && out_len)) {             /* the reference would fault */
        errno = EINVAL;
        return 0;
    }
    if (!out_data) out_data = &none;                      /* out_len 0: nothing is written */
    uint64_t zero = 0;
    uint32_t res = 0;
    int32_t err = 0;
    const int rc = host_batch_rc(false, (const uint8_t *)in_data, &zero, &in_len, (uint8_t *)out_data, &zero,
                                 &out_len, &res, &err, 1);
    if (rc != LZF_GPU_OK) {
        errno = EIO;
        return 0;
    }
    if (!res) errno = err ? err : EINVAL;
    return res;
}

int lzf_gpu_compress_batch(const uint8_t *in, const uint64_t *in_off, const uint32_t *in_len,
                           uint8_t *out, const uint64_t *out_off, const uint32_t *out_cap,
                           uint32_t *out_len, uint32_t count, uint32_t max_in_len, void *stream)
{
    if (!count || !in || !in_off || !in_len || !out || !out_off || !out_cap || !out_len) return LZF_GPU_EARG;
    if (max_in_len > LZF_GPU_MAX_VALUE) return LZF_GPU_EARG;
    int rc = current_device_ok();
    if (rc) return rc;
    if (!max_in_len)                  /* every value empty: out_len 0 each (src/lzf_c.c:131) */
        return hipMemsetAsync(out_len, 0, (size_t)count * sizeof(uint32_t), (hipStream_t)stream) == hipSuccess
                   ? LZF_GPU_OK
                   : LZF_GPU_ELAUNCH;
    LzfBatch b{in, in_off, in_len, out, out_off, out_cap, out_len, nullptr, count, max_in_len};
    const hipError_t e = launch_compress(b, (hipStream_t)stream);
    return e == hipSuccess ? LZF_GPU_OK : code_of(e);
}

int lzf_gpu_decompress_batch(const uint8_t *in, const uint64_t *in_off, const uint32_t *in_len,
                             uint8_t *out, const uint64_t *out_off, const uint32_t *out_cap,
                             uint32_t *out_len, int32_t *err, uint32_t count,
                             uint32_t max_out_cap, void *stream)
{
    if (!count || !in || !in_off || !in_len || !out || !out_off || !out_cap || !out_len || !err)
        return LZF_GPU_EARG;
    int rc = current_device_ok();
    if (rc) return rc;
    LzfBatch b{in, in_off, in_len, out, out_off, out_cap, out_len, err, count, max_out_cap};
    const hipError_t e = launch_decompress(b, (hipStream_t)stream);
    return e == hipSuccess ? LZF_GPU_OK : code_of(e);
}

void lzf_gpu_release(void)
{
    for (Scratch &S : g_scratch) {
        std::lock_guard<std::mutex> lk(S.mu);
        scratch_free(S);
    }
    try {
        ctx().release();
    } catch (const LzfFail &) {
    }
}

int lzf_gpu_synth_fill(int kind, uint64_t seed, uint64_t first, uint64_t stride, uint32_t count,
                       uint32_t n, uint8_t *out, void *stream)
{
    if (!count || !n || !out || kind < 0) return LZF_GPU_EARG;
    int rc = current_device_ok();
    if (rc) return rc;
    return lzf_launch_synth(kind, seed, first, stride, count, n, out, (hipStream_t)stream) ==
                   hipSuccess
               ? LZF_GPU_OK
               : LZF_GPU_ELAUNCH;
}

int lzf_host_compress_batch(const uint8_t *in, const uint64_t *in_off, const uint32_t *in_len,
                            uint8_t *out, const uint64_t *out_off, const uint32_t *out_cap,
                            uint32_t *out_len, uint32_t count)
{
    return host_batch_rc(true, in, in_off, in_len, out, out_off, out_cap, out_len, nullptr, count);
}

int lzf_host_decompress_batch(const uint8_t *in, const uint64_t *in_off, const uint32_t *in_len,
                              uint8_t *out, const uint64_t *out_off, const uint32_t *out_cap,
                              uint32_t *out_len, int32_t *err, uint32_t count)
{
    return host_batch_rc(false, in, in_off, in_len, out, out_off, out_cap, out_len, err, count);
}

int lzf_gpu_decoded_size_batch(const uint8_t *in, const uint64_t *in_off, const uint32_t *in_len,
                               uint32_t *out_size, int32_t *err, uint32_t count, uint32_t out_limit, void *stream)
{
    if (!count || !in || !in_off || !in_len || !out_size || !err) return LZF_GPU_EARG;
    int rc = current_device_ok();
    if (rc) return rc;
    return lzf_launch_dsize(in, in_off, in_len, out_size, err, count, out_limit, (hipStream_t)stream) == hipSuccess
               ? LZF_GPU_OK
               : LZF_GPU_ELAUNCH;
}

int lzf_host_decoded_size_batch(const uint8_t *in, const uint64_t *in_off, const uint32_t *in_len,
                                uint32_t *out_size, int32_t *err, uint32_t count, uint32_t out_limit)
{
    return host_dsize(in, in_off, in_len, out_size, err, count, out_limit);
}

uint64_t lzf_gpu_kv_frame_work_size(uint32_t count)
{
    return lzf_frame_work_bytes(count);
}

int lzf_gpu_kv_frame(const uint8_t *keys, const uint64_t *key_off, const uint32_t *key_len,
                     const uint8_t *vals, const uint64_t *val_off, const uint32_t *val_size,
                     const uint8_t *enc, const uint32_t *val_len, uint32_t count,
                     uint32_t elements, uint32_t max_val_len, int reply_header,
                     uint8_t *frame, uint64_t max_response, uint64_t *frame_len, void *work,
                     void *stream)
{
    if (!count || !keys || !key_off || !key_len || !vals || !val_off || !val_size || !enc ||
        !val_len || !frame || !frame_len || !work)
        return LZF_GPU_EARG;
    if (max_val_len > LZF_GPU_MAX_VALUE) return LZF_GPU_EARG;
    int rc = current_device_ok();
    if (rc) return rc;
    LzfFrameArgs a{};
    a.keys = keys; a.key_off = key_off; a.key_len = key_len;
    a.vals = vals; a.val_off = val_off; a.val_size = val_size;
    a.enc = enc; a.val_len = val_len;
    a.count = count; a.elements = elements; a.max_val_len = max_val_len ? max_val_len : 1u;
    a.reply_header = reply_header;
    a.max_response = max_response;
    a.frame = frame; a.frame_len = frame_len;
    lzf_frame_carve(a, work);
    return lzf_launch_frame(a, (hipStream_t)stream, launch_decompress) == hipSuccess ? LZF_GPU_OK
                                                                                    : LZF_GPU_ELAUNCH;
}

int lzf_gpu_selfcheck(void)
{
    int rc = current_device_ok();
    if (rc) return rc;
    const int st = lds_order_state(true);
    return st == 1 ? 1 : st == -1 ? 0 : LZF_GPU_ELAUNCH;
}

int lzf_gpu_lds_order_probe(void)
{
    int rc = current_device_ok();
    if (rc) return rc;
    int dev = 0;
    if (hipGetDevice(&dev) != hipSuccess) return LZF_GPU_ENODEV;
    return lzf_lds_order_check(dev);
}

const char *lzf_gpu_kernel_info(void)
{
    static thread_local std::string s;
    switch (kernel_gen()) {
#ifdef LZF_DIAG
    case GEN_SERIAL: s = "compress=serial decompress=serial"; break;
#endif
    case GEN_WINDOW:
        s = std::string("compress=") + lzf_compress_kernel_name() + " decompress=" +
            lzf_decompress_kernel_name();
        break;
#ifdef LZF_DIAG
    case GEN_WTAB:
        s = std::string("compress=wtab(cand_q1+wparse; window64 past 64 KiB) decompress=") +
            lzf_decompress_kernel_name();
        break;
#endif
    case GEN_TABLE_ONLY:
        s = std::string("compress=table(cand_table+parse_rec; window64 past 64 KiB or below ") +
            std::to_string(lane_min_count(4096u)) + " values of <= 4 KiB / " +
            std::to_string(lane_min_count(8192u)) + " of <= 8 KiB / " +
            std::to_string(lane_min_count(16384u)) + " of <= 16 KiB / " +
            std::to_string(lane_min_count(65536u)) + " of <= 64 KiB) decompress=" +
            (lane_decoder() ? "lane" : lzf_decompress_kernel_name());
        break;
    case GEN_LANE:
        s = std::string("compress=lane(") + lzf_lane_cand_name() + "+parse_lane; window64 past 64 KiB or below " +
            std::to_string(lane_min_count(4096u)) + " values of <= 4 KiB / " +
            std::to_string(lane_min_count(8192u)) + " of <= 8 KiB / " +
            std::to_string(lane_min_count(16384u)) + " of <= 16 KiB / " +
            std::to_string(lane_min_count(65536u)) + " of <= 64 KiB) decompress=" +
            (lane_decoder() ? "lane" : lzf_decompress_kernel_name());
        break;
    default:
        s = std::string("compress=lane(") + lzf_lane_cand_name() + "+parse_lane) up to " +
            std::to_string(LANE_DEFAULT_MAX / 1024u) + " KiB, table(cand_table+parse_rec) up to 64 KiB; window64 past 64 KiB or below " +
            std::to_string(lane_min_count(4096u)) + " values of <= 4 KiB / " +
            std::to_string(lane_min_count(8192u)) + " of <= 8 KiB / " +
            std::to_string(lane_min_count(16384u)) + " of <= 16 KiB / " +
            std::to_string(lane_min_count(65536u)) + " of <= 64 KiB) decompress=" +
            (lane_decoder() ? "lane" : lzf_decompress_kernel_name());
        break;
    }
    {
        const int st = lds_order_state(false);
        s += std::string(" lds_order=") + (st == 1 ? "held" : st == -1 ? "violated(compress->window64)"
                                           : st == -2 ? "probe-failed(retried)" : "unchecked");
        if (g_last_chunks) s += " scratch_chunks=" + std::to_string(g_last_chunks);
    }
    return s.c_str();
}

}  // extern "C"
