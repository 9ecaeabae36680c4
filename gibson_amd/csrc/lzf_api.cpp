/*
 * lzf_api.cpp -- the device side of liblzf_hip.so's C-ABI.
 *
 * The kernel routing (which generation compresses a batch, which decoder
 * decodes it), the per-device compress scratch and the LDS lane-order
 * self-check, and the device-pointer calls of include/lzf_gpu.h.  The
 * host-memory calls -- the drop-in pair of include/lzf.h (src/lzf.h:76-78,
 * 95-97) and the lzf_host_* batches -- are in lzf_host.cpp and launch
 * through lzf_route_compress / lzf_route_decompress below.  There is no CPU
 * codec in this library: every call runs the HIP kernels.  Failures never
 * abort (a server must survive a transient HIP error): the batch calls
 * return a negative LZF_GPU_E* code (LZF_GPU_ENODEV without a device).
 */
#include <errno.h>
#include <stdio.h>
#include <stdlib.h>
#include <string.h>

#include <algorithm>
#include <chrono>
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
/* a probe that could not run is retried no sooner than this (a backoff
 * doubling from 100 ms to 10 s, so a lasting failure -- memory pressure, a
 * caller capturing a graph -- does not cost every compress call a probe
 * under the mutex) */
std::chrono::steady_clock::time_point g_order_retry[64];
std::chrono::milliseconds g_order_backoff[64];
std::mutex g_order_mu;

int lds_order_state(bool run)
{
    int dev = 0;
    if (hipGetDevice(&dev) != hipSuccess || dev < 0 || dev >= 64) return -2;
    std::lock_guard<std::mutex> lk(g_order_mu);
    const auto now = std::chrono::steady_clock::now();
    if (!g_order[dev] && run && (g_order_last[dev] != -2 || now >= g_order_retry[dev])) {
        const char *f = getenv("LZF_GPU_FORCE_ORDER_FAIL");
        const int bad = (f && *f == '1') ? 1 : lzf_lds_order_check(dev);
        g_order_last[dev] = bad == 0 ? 1 : bad > 0 ? -1 : -2;
        if (bad >= 0) {
            g_order[dev] = g_order_last[dev];
        } else {
            auto &b = g_order_backoff[dev];
            b = b.count() ? std::min(b * 2, std::chrono::milliseconds(10000)) : std::chrono::milliseconds(100);
            g_order_retry[dev] = now + b;
        }
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
    /* this scratch's share of the cap: 1 for the device's, NSLOT for each
     * chunk slot of the registered host pipeline, whose launches run side by
     * side and keep their buffers between calls -- together they stay within
     * one cap instead of taking half of what each one finds free */
    unsigned share = 1;
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
size_t scratch_limit(size_t held, unsigned share = 1)
{
    if (share < 1) share = 1;
    const char *e = getenv("LZF_GPU_SCRATCH_MB");
    if (e) {
        unsigned long long mb = strtoull(e, nullptr, 10);
        if (mb < 1) mb = 1;
        return ((size_t)mb << 20) / share;
    }
    size_t fr = 0, tot = 0;
    if (hipMemGetInfo(&fr, &tot) != hipSuccess) return ((size_t)40 << 30) / share;
    /* held: this scratch's own buffer, which a regrow gives back first; the
     * slot scratches' shares are of the device's total, so buffers the other
     * slots already hold do not shrink the next one's share */
    size_t lim = share == 1 ? (fr + held) / 2 : tot / (2 * (size_t)share);
    if (share > 1 && lim > fr + held) lim = fr + held;
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

/* own: a caller's private scratch (the host pipelines' slots, so their
 * chunks' compress launches can run side by side), else the device's */
hipError_t lane_compress(const LzfBatch &b, hipStream_t s, ScratchUser who, Scratch *own = nullptr,
                         const LzfParts *parts = nullptr)
{
    const bool table = who == SU_TABLE;
    int dev = 0;
    hipError_t e = hipGetDevice(&dev);
    if (e != hipSuccess) return e;
    Scratch &S = own ? *own : g_scratch[dev & 63];
    std::lock_guard<std::mutex> lk(S.mu);
#ifdef LZF_DIAG
    const size_t per = who == SU_WTAB ? lzf_wtab_scratch_per_value(b.max_len)
                       : table        ? lzf_table_scratch_per_value(b.max_len)
                                      : lzf_lane_scratch_per_value(b.max_len);
#else
    const size_t per = table ? lzf_table_scratch_per_value(b.max_len) : lzf_lane_scratch_per_value(b.max_len);
#endif
    size_t want = per * (size_t)b.count + 512;
    const size_t lim = scratch_limit(S.cap, S.share);
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
        e = lzf_launch_compress_table(b, s, S.p, use, &g_last_chunks, parts);
    }
#ifdef LZF_DIAG
    else if (who == SU_WTAB) {
        e = lzf_launch_compress_wtab(b, s, S.p, use, &g_last_chunks);
    }
#endif
    else {
        /* the lane generation takes the batch whole: every part in first */
        for (uint32_t p = 0; parts && p < parts->n; p++)
            if ((e = hipStreamWaitEvent(s, parts->ev[p], 0)) != hipSuccess) return e;
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

/* bulk: the caller runs several launches side by side (the host-memory
 * pipeline), so the per-launch floor of the parse overlaps and the batch
 * threshold below which window64 wins alone does not apply */
hipError_t launch_compress(const LzfBatch &b, hipStream_t s, Scratch *own = nullptr, bool bulk = false,
                           const LzfParts *parts = nullptr)
{
    const KernelGen g = kernel_gen();
    /* inputs in parts: a route that takes the batch whole waits for all */
    const bool routed_default = g == GEN_TABLE && lds_order_ok() && lzf_table_compress_supported(b.max_len);
    if (parts && !routed_default)
        for (uint32_t p = 0; p < parts->n; p++) {
            const hipError_t e = hipStreamWaitEvent(s, parts->ev[p], 0);
            if (e != hipSuccess) return e;
        }
    if (!routed_default) parts = nullptr;
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
        if ((!bulk && b.count < lane_min_count(b.max_len)) || !lzf_table_compress_supported(b.max_len)) {
            for (uint32_t p = 0; parts && p < parts->n; p++) {
                const hipError_t e = hipStreamWaitEvent(s, parts->ev[p], 0);
                if (e != hipSuccess) return e;
            }
            return lzf_launch_compress(b, s);
        }
        /* the lane generation where its kernel 1 takes the batch (a
         * diagnostic LZF_GPU_CAND=small stops at 4 KiB), else the table one --
         * unless the scratch cap splits the table generation into more chunks
         * than the lane generation (half the scratch per value): every chunk
         * pays the parse's per-launch floor, so the chunk count decides
         * (configs[2] under a 16 GiB cap: table 5 chunks 441 ms, lane 3 chunks
         * 335 ms; 8 GiB: 712 / 488; uncapped table 190 vs lane 214,
         * profiles/r05/cap/) */
        {
            bool lane = b.max_len <= LANE_DEFAULT_MAX && lzf_lane_compress_supported(b.max_len);
            if (!lane && lzf_lane_compress_supported(b.max_len)) {
                int dev = 0;
                if (hipGetDevice(&dev) == hipSuccess) {
                    Scratch &S = own ? *own : g_scratch[dev & 63];
                    size_t held;
                    unsigned share;
                    {
                        /* another thread's lane_compress may be regrowing it */
                        std::lock_guard<std::mutex> lk(S.mu);
                        held = S.cap;
                        share = S.share;
                    }
                    const size_t lim = scratch_limit(held, share);
                    const uint64_t need_t = (uint64_t)b.count * lzf_table_scratch_per_value(b.max_len);
                    const uint64_t need_l = (uint64_t)b.count * lzf_lane_scratch_per_value(b.max_len);
                    lane = (need_t + lim - 1) / lim > (need_l + lim - 1) / lim;
                }
            }
            return lane_compress(b, s, lane ? SU_LANE : SU_TABLE, own, parts);
        }
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

int code_of(hipError_t e)
{
    if (e == hipErrorOutOfMemory || e == hipErrorMemoryAllocation) return LZF_GPU_ENOMEM;
    if (e == hipErrorNoDevice || e == hipErrorInvalidDevice) return LZF_GPU_ENODEV;
    return LZF_GPU_ELAUNCH;
}

}  // namespace

/* the routed launches and the scratch, for the host-memory paths (lzf_host.cpp) */
hipError_t lzf_route_compress(const LzfBatch &b, hipStream_t s) { return launch_compress(b, s); }
hipError_t lzf_route_decompress(const LzfBatch &b, hipStream_t s) { return launch_decompress(b, s); }
uint32_t lzf_route_min_count(uint32_t max_len) { return lane_min_count(max_len); }
bool lzf_device_ok(int dev) { return device_ok(dev); }
hipError_t lzf_route_compress_window(const LzfBatch &b, hipStream_t s) { return lzf_launch_compress(b, s); }
bool lzf_route_default(void) { return kernel_gen() == GEN_TABLE && lds_order_ok(); }
hipError_t lzf_route_compress_bulk(const LzfBatch &b, hipStream_t s, void *scratch, const LzfParts *parts)
{
    return launch_compress(b, s, (Scratch *)scratch, true, parts);
}
void *lzf_scratch_create(unsigned share)
{
    Scratch *S = new Scratch();
    S->share = share ? share : 1u;
    return S;
}
void lzf_scratch_destroy(void *scratch)
{
    Scratch *S = (Scratch *)scratch;
    if (!S) return;
    {
        std::lock_guard<std::mutex> lk(S->mu);
        scratch_free(*S);
        if (S->ev) (void)hipEventDestroy(S->ev);
    }
    delete S;
}
void lzf_scratch_release(void *scratch)
{
    Scratch *S = (Scratch *)scratch;
    if (!S) return;
    std::lock_guard<std::mutex> lk(S->mu);
    scratch_free(*S);
}
void lzf_scratch_release_all(void)
{
    for (Scratch &S : g_scratch) {
        std::lock_guard<std::mutex> lk(S.mu);
        scratch_free(S);
    }
}

extern "C" {

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
