/*
 * lzf_host.cpp -- the host-memory side of liblzf_hip.so.
 *
 * The drop-in pair of include/lzf.h (src/lzf.h:76-78, 95-97, replacing
 * src/lzf_c.c:98 and src/lzf_d.c:55) and the host-memory batch calls of
 * include/lzf_gpu.h.  Gibson's path starts in host memory -- the client's
 * request buffer (src/server.c:180) on the way in, the trie-resident value
 * (src/query.c:409) on the way out -- so these calls move values over PCIe,
 * run the routed kernels (lzf_api.cpp) and bring the results back.
 *
 * Devices.  Gibson is one process with one event loop
 * (src/net.c:578-589, README.md:13); the only place it can use several GPUs
 * is this library.  LZF_GPU_DEVICES names them ("0,1,2,3", "all"; a device
 * may repeat: "0,0" runs two contexts on device 0).  A host batch sends value
 * i to entry i mod G; each entry has a persistent worker thread with its own
 * non-blocking streams, pinned staging and, on its device, the shared compress
 * scratch.  The worker binds itself to its device's NUMA node (read from
 * sysfs through the PCI bus id) before it allocates anything, so its pinned
 * staging is node-local.  Results land at index i; a failing entry makes the
 * batch return its LZF_GPU_E* code, never an abort.  Unset, LZF_GPU_DEVICE
 * (default 0) is the one device and batches run on the calling thread.
 *
 * Moving bytes.  Two paths, same results:
 *  - registered (lzf_host_register): the caller's arenas are page-locked and
 *    mapped, so the GPU reads each value from, and writes each stream to,
 *    the caller's memory itself (lzf_hostio.hip) -- or the DMA engines copy
 *    runs of adjacent values -- and the CPU touches only descriptors;
 *  - staged (anything else): the CPU packs values into pinned staging and
 *    unpacks the results (several threads), in a two-slot chunk pipeline for
 *    large batches.
 */
#include <ctype.h>
#include <errno.h>
#include <pthread.h>
#include <sched.h>
#include <stdio.h>
#include <stdlib.h>
#include <string.h>
#include <sys/syscall.h>
#include <unistd.h>

#include <chrono>
#include <condition_variable>
#include <deque>
#include <functional>
#include <iterator>
#include <map>
#include <memory>
#include <mutex>
#include <string>
#include <thread>
#include <vector>

#include "lzf_internal.h"
#include "../../include/lzf.h"
#include "../../include/lzf_gpu.h"

namespace {

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
        if (prev != dev) check(hipSetDevice(dev), "hipSetDevice");
    }
    ~DeviceGuard()
    {
        int cur = -1;
        if (prev >= 0 && hipGetDevice(&cur) == hipSuccess && cur != prev) (void)hipSetDevice(prev);
    }
};

/* ---- the device plan (LZF_GPU_DEVICES) ---------------------------------- */

struct Plan {
    std::vector<int> dev;
    int rc = LZF_GPU_OK;
};

const Plan &plan()
{
    static const Plan p = [] {
        Plan q;
        const char *e = getenv("LZF_GPU_DEVICES");
        if (!e || !*e) {
            const char *d = getenv("LZF_GPU_DEVICE");
            q.dev.push_back(d ? atoi(d) : 0);
            return q;
        }
        int visible = 0;
        if (hipGetDeviceCount(&visible) != hipSuccess) visible = 0;
        int buf[64];
        const int n = lzf_gpu_parse_device_list(e, visible, buf, 64);
        if (n <= 0) {
            fprintf(stderr, "liblzf_hip: LZF_GPU_DEVICES=\"%s\" names no usable device (%d visible)\n", e, visible);
            q.rc = LZF_GPU_ENODEV;
            q.dev.push_back(0);
            return q;
        }
        for (int k = 0; k < n; k++) {
            if (!lzf_device_ok(buf[k])) {
                fprintf(stderr, "liblzf_hip: LZF_GPU_DEVICES entry %d (device %d) is not a gfx950\n", k, buf[k]);
                q.rc = LZF_GPU_ENODEV;
            }
            q.dev.push_back(buf[k]);
        }
        return q;
    }();
    return p;
}

/* ---- NUMA: the node of a device and binding a thread to it --------------- */

bool parse_cpulist(const char *s, cpu_set_t *set)
{
    CPU_ZERO(set);
    bool any = false;
    while (*s) {
        char *end;
        long a = strtol(s, &end, 10);
        if (end == s) break;
        long b = a;
        s = end;
        if (*s == '-') {
            b = strtol(s + 1, &end, 10);
            s = end;
        }
        for (long c = a; c <= b && c < CPU_SETSIZE; c++) {
            CPU_SET((int)c, set);
            any = true;
        }
        if (*s == ',') s++;
        else break;
    }
    return any;
}

/* the device's NUMA node from sysfs (-1: unknown) and that node's CPUs */
int device_numa(int dev, cpu_set_t *cpus)
{
    CPU_ZERO(cpus);
    char bus[64] = {0};
    if (hipDeviceGetPCIBusId(bus, sizeof bus, dev) != hipSuccess) return -1;
    for (char *c = bus; *c; c++) *c = (char)tolower((unsigned char)*c);
    const std::string base = std::string("/sys/bus/pci/devices/") + bus;
    int node = -1;
    if (FILE *f = fopen((base + "/numa_node").c_str(), "r")) {
        if (fscanf(f, "%d", &node) != 1) node = -1;
        fclose(f);
    }
    if (FILE *f = fopen((base + "/local_cpulist").c_str(), "r")) {
        char line[4096] = {0};
        if (fgets(line, sizeof line, f)) parse_cpulist(line, cpus);
        fclose(f);
    }
    return node;
}

/* Pin the calling thread to the node's CPUs that this process may use and
 * prefer the node for its memory (set_mempolicy MPOL_PREFERRED; pinned
 * staging is then allocated with hipHostMallocNumaUser).  False when the
 * node is unknown or none of its CPUs is in the process's affinity set. */
bool bind_to_node(int node, const cpu_set_t &local)
{
    if (node < 0 || node >= 1024) return false;
    cpu_set_t allowed, both;
    if (sched_getaffinity(0, sizeof allowed, &allowed) != 0) return false;
    CPU_AND(&both, &allowed, &local);
    if (CPU_COUNT(&both) == 0) return false;
    if (pthread_setaffinity_np(pthread_self(), sizeof both, &both) != 0) return false;
    unsigned long mask[1024 / (8 * sizeof(unsigned long))] = {0};
    mask[node / (8 * sizeof(unsigned long))] |= 1ul << (node % (8 * sizeof(unsigned long)));
    const long MPOL_PREFERRED_ = 1;
    return syscall(SYS_set_mempolicy, MPOL_PREFERRED_, mask, (unsigned long)1024) == 0;
}

/* ---- per-thread contexts ------------------------------------------------- */

/* Growable device / pinned buffers of one context. */
struct Buf {
    void *p = nullptr;
    size_t cap = 0;
    bool pinned = false;
    unsigned flags = hipHostMallocDefault;
    void *get(size_t need)
    {
        if (need == 0) need = 1;
        if (need <= cap) return p;
        size_t want = need + need / 4 + 256;
        if (p) { pinned ? (void)hipHostFree(p) : (void)hipFree(p); }
        p = nullptr;
        cap = 0;
        hipError_t e = pinned ? hipHostMalloc(&p, want, flags) : hipMalloc(&p, want);
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

/* One stage of a chunk pipeline: its own stream, pinned and device buffers,
 * and the chunk it holds until its results are taken. */
struct Slot {
    hipStream_t stream = nullptr;
    hipEvent_t done = nullptr;
    Buf d_in, d_out, d_meta;
    Buf h_in{nullptr, 0, true}, h_out{nullptr, 0, true}, h_meta{nullptr, 0, true};
    void *scratch = nullptr;       /* the slot's own compress scratch (registered path) */
    hipEvent_t in_done = nullptr;  /* the chunk's inputs are on the device (registered path) */
    hipEvent_t out_done = nullptr; /* the chunk's outputs are in host memory (registered path) */
    uint32_t first = 0, count = 0;
    bool busy = false;
};
constexpr uint32_t NSLOT = 3;      /* registered path: chunks in flight */
constexpr uint32_t TAIL_MAX = 4;   /* tail mode: window64 chunks (at most), each with its own slot */
constexpr uint32_t NSLOT_ALL = 1u + TAIL_MAX;
#ifndef CHAIN_OUT
#define CHAIN_OUT 1                /* registered path: chunk outputs cross the bus in order */
#endif

struct Ctx {
    int dev = 0;
    bool ok = false;
    bool numa_bound = false;
    hipStream_t stream = nullptr;
    Buf d_in, d_out, d_meta;
    /* registered compress, tail mode: the routed chunk's inputs in parts on
     * their own stream (one event per part) */
    hipStream_t in_stream = nullptr;
    std::vector<hipEvent_t> in_ev;
    Buf h_in{nullptr, 0, true}, h_out{nullptr, 0, true}, h_meta{nullptr, 0, true};
    Slot slot[NSLOT_ALL];
    Ctx(int device, bool bound) : dev(device), numa_bound(bound)
    {
        int n = 0;
        if (hipGetDeviceCount(&n) != hipSuccess || dev < 0 || dev >= n || !lzf_device_ok(dev)) {
            fprintf(stderr, "liblzf_hip: no gfx950 device %d (devices: %d); the codec runs on the GPU only\n", dev,
                    n);
            return;
        }
        const unsigned fl = bound ? (unsigned)hipHostMallocNumaUser : (unsigned)hipHostMallocDefault;
        for (Buf *b : {&h_in, &h_out, &h_meta}) b->flags = fl;
        for (auto &sl : slot)
            for (Buf *b : {&sl.h_in, &sl.h_out, &sl.h_meta}) b->flags = fl;
        int prev = -1;
        (void)hipGetDevice(&prev);
        (void)hipSetDevice(dev);
        ok = hipStreamCreateWithFlags(&stream, hipStreamNonBlocking) == hipSuccess;
        if (prev >= 0 && prev != dev) (void)hipSetDevice(prev);
    }
    /* this context's buffers (at its thread's exit, or lzf_gpu_release) */
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
            lzf_scratch_release(sl.scratch);
            sl.busy = false;
        }
        if (in_stream) (void)hipStreamSynchronize(in_stream);
        for (Buf *b : {&d_in, &d_out, &d_meta, &h_in, &h_out, &h_meta}) b->release();
        if (prev >= 0 && prev != dev) (void)hipSetDevice(prev);
    }
    /* after a failure: wait for what is in flight, so the buffers are free */
    void quiesce()
    {
        if (!ok) return;
        if (stream) (void)hipStreamSynchronize(stream);
        if (in_stream) (void)hipStreamSynchronize(in_stream);
        for (auto &sl : slot) {
            if (sl.stream) (void)hipStreamSynchronize(sl.stream);
            sl.busy = false;
        }
        (void)hipGetLastError();
    }
    ~Ctx()
    {
        release();
        for (auto &sl : slot) lzf_scratch_destroy(sl.scratch);
        for (hipEvent_t e : in_ev) (void)hipEventDestroy(e);
        if (in_stream) (void)hipStreamDestroy(in_stream);
    }
};

/* the calling thread's context, on the plan's first device, made on its
 * first host-memory call (a thread that only uses the device-pointer calls
 * never makes one: no stream or staging on a device it does not use) */
thread_local std::unique_ptr<Ctx> t_caller;
Ctx &caller_ctx()
{
    if (!t_caller) t_caller.reset(new Ctx(plan().dev[0], false));
    if (!t_caller->ok) throw LzfFail{LZF_GPU_ENODEV};
    return *t_caller;
}

/* ---- registered host ranges (lzf_host_register) --------------------------- */

/* every distinct device of the plan maps [ptr, ptr + len): a device address
 * for its first and last byte, on that device (LZF_GPU_ENODEV otherwise; the
 * registration is then undone).  LZF_GPU_FORCE_MAP_FAIL=<device> makes that
 * device's check fail (the tests of the refusal). */
int register_check_devices(const std::vector<int> &devs, const void *ptr, uint64_t len)
{
    const char *ff = getenv("LZF_GPU_FORCE_MAP_FAIL");
    const int force = ff && *ff ? atoi(ff) : -1;
    std::vector<int> seen;
    for (int d : devs) {
        bool dup = false;
        for (int x : seen) dup = dup || x == d;
        if (dup) continue;
        seen.push_back(d);
        if (hipSetDevice(d) != hipSuccess) {
            (void)hipGetLastError();
            return LZF_GPU_ENODEV;
        }
        void *p0 = nullptr, *p1 = nullptr;
        const bool ok = hipHostGetDevicePointer(&p0, (void *)ptr, 0) == hipSuccess &&
                        hipHostGetDevicePointer(&p1, (void *)((const uint8_t *)ptr + len - 1), 0) == hipSuccess &&
                        p0 && (uintptr_t)p1 - (uintptr_t)p0 == len - 1 && d != force;
        if (!ok) {
            (void)hipGetLastError();
            fprintf(stderr, "liblzf_hip: registered range not mapped on device %d\n", d);
            return LZF_GPU_ENODEV;
        }
    }
    return LZF_GPU_OK;
}

std::mutex g_reg_mu;
std::map<uintptr_t, uintptr_t> g_reg;      /* start -> end of each registered range */

/* true when [lo, hi) lies inside one registered range */
bool is_registered(uintptr_t lo, uintptr_t hi)
{
    std::lock_guard<std::mutex> lk(g_reg_mu);
    auto it = g_reg.upper_bound(lo);
    if (it == g_reg.begin()) return false;
    --it;
    return lo >= it->first && hi <= it->second;
}

/* ---- one host batch ------------------------------------------------------ */

/* the caller's arrays of one host-memory call */
struct HostArgs {
    bool compress;
    const uint8_t *in;
    const uint64_t *in_off;
    const uint32_t *in_len;
    uint8_t *out;
    const uint64_t *out_off;
    const uint32_t *out_cap;
    uint32_t *out_len;
    int32_t *err;
};

/* value k of a sub-batch is the caller's value first + k * stride */
struct View {
    uint32_t first = 0, stride = 1, count = 0;
    uint32_t at(uint32_t k) const { return first + k * stride; }
};

/* a 0-length stream still reads its first control byte (src/lzf_d.c:64-66) */
inline uint32_t in_extent(const HostArgs &a, uint32_t i)
{
    return a.in_len[i] ? a.in_len[i] : (a.compress ? 0u : 1u);
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

hipError_t launch(const HostArgs &a, const LzfBatch &b, hipStream_t s)
{
    return a.compress ? lzf_route_compress(b, s) : lzf_route_decompress(b, s);
}

void make_slot_streams(Ctx &c)
{
    for (auto &sl : c.slot) {
        if (!sl.stream) check(hipStreamCreateWithFlags(&sl.stream, hipStreamNonBlocking), "hipStreamCreate");
        if (!sl.done) check(hipEventCreateWithFlags(&sl.done, hipEventDisableTiming), "hipEventCreate");
        if (!sl.scratch) sl.scratch = lzf_scratch_create(NSLOT);   /* the slots share one cap */
        if (!sl.in_done) check(hipEventCreateWithFlags(&sl.in_done, hipEventDisableTiming), "hipEventCreate");
        if (!sl.out_done) check(hipEventCreateWithFlags(&sl.out_done, hipEventDisableTiming), "hipEventCreate");
        sl.busy = false;
    }
}

/* Staged, chunked: values in chunks through two slots on two streams.  The
 * CPU packs chunk k+1's values into pinned staging (several threads) while
 * chunk k moves over PCIe and runs; results are unpacked once a slot comes
 * round again.  Each chunk's values are packed (inputs back to back, outputs
 * at their caps back to back), so only their bytes cross the bus. */
void host_batch_staged(Ctx &c, const HostArgs &a, const View &v, uint64_t chunk_in, uint64_t chunk_out)
{
    const uint32_t threads = host_threads();
    make_slot_streams(c);
    const size_t mrec = 2 * sizeof(uint64_t) + 4 * sizeof(uint32_t);
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
                const uint32_t i = v.at(sl.first + k);
                a.out_len[i] = m_out_len[k];
                if (a.err) a.err[i] = m_err[k];
                if (m_out_len[k]) memcpy(a.out + a.out_off[i], h_out + m_out_off[k], m_out_len[k]);
            }
        });
        sl.busy = false;
    };
    uint32_t k0 = 0, round = 0;
    while (k0 < v.count) {
        uint64_t bin = 0, bout = 0;
        uint32_t k1 = k0, max_len = 0;
        while (k1 < v.count) {
            const uint32_t i = v.at(k1);
            const uint64_t li = in_extent(a, i) ? in_extent(a, i) : 1u;
            if (k1 > k0 && (bin + li > chunk_in || bout + a.out_cap[i] > chunk_out)) break;
            bin += li;
            bout += a.out_cap[i];
            const uint32_t l = a.compress ? a.in_len[i] : a.out_cap[i];
            if (l > max_len) max_len = l;
            k1++;
        }
        Slot &sl = c.slot[round & 1u];      /* two slots: CPU packing is the bound */
        drain(sl);
        const uint32_t n = k1 - k0;
        uint8_t *h_in = (uint8_t *)sl.h_in.get(bin);
        uint8_t *h_meta = (uint8_t *)sl.h_meta.get((size_t)n * mrec);
        uint8_t *d_in = (uint8_t *)sl.d_in.get(bin);
        uint8_t *d_out = (uint8_t *)sl.d_out.get(bout);
        uint8_t *d_meta = (uint8_t *)sl.d_meta.get((size_t)n * mrec);
        sl.h_out.get(bout);
        uint64_t *m_in_off = (uint64_t *)h_meta, *m_out_off = m_in_off + n;
        uint32_t *m_in_len = (uint32_t *)(m_out_off + n), *m_out_cap = m_in_len + n;
        {
            uint64_t x = 0, y = 0;
            for (uint32_t j = 0; j < n; j++) {
                const uint32_t i = v.at(k0 + j);
                m_in_off[j] = x;
                m_out_off[j] = y;
                m_in_len[j] = a.in_len[i];
                m_out_cap[j] = a.out_cap[i];
                x += in_extent(a, i) ? in_extent(a, i) : 1u;
                y += a.out_cap[i];
            }
        }
        parallel_ranges(n, threads, [&](uint32_t lo, uint32_t hi) {
            for (uint32_t j = lo; j < hi; j++) {
                const uint32_t i = v.at(k0 + j);
                if (in_extent(a, i)) memcpy(h_in + m_in_off[j], a.in + a.in_off[i], in_extent(a, i));
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
        check(launch(a, b, sl.stream), "kernel launch");
        check(hipMemcpyAsync(h_meta + res_off, d_meta + res_off, (size_t)n * mrec - res_off, hipMemcpyDeviceToHost,
                             sl.stream),
              "hipMemcpyAsync");
        check(hipMemcpyAsync(sl.h_out.p, d_out, bout, hipMemcpyDeviceToHost, sl.stream), "hipMemcpyAsync");
        check(hipEventRecord(sl.done, sl.stream), "hipEventRecord");
        sl.first = k0;
        sl.count = n;
        sl.busy = true;
        k0 = k1;
        round++;
    }
    drain(c.slot[round & 1u]);
    drain(c.slot[(round + 1u) & 1u]);
}

/* Staged, one piece (small batches, and decodes whose caps are far above
 * their inputs -- the drop-in lzf_decompress at out_len = maxrequestsize):
 * after the kernel only the produced bytes come back. */
void host_batch_small(Ctx &c, const HostArgs &a, const View &v)
{
    const uint32_t n = v.count;
    uint64_t bin = 0, bout = 0;
    uint32_t max_len = 0;
    for (uint32_t k = 0; k < n; k++) {
        const uint32_t i = v.at(k);
        bin += in_extent(a, i) ? in_extent(a, i) : 1u;
        bout += a.out_cap[i];
        const uint32_t l = a.compress ? a.in_len[i] : a.out_cap[i];
        if (l > max_len) max_len = l;
    }
    const size_t meta_bytes = (size_t)n * (2 * sizeof(uint64_t) + 4 * sizeof(uint32_t));
    uint8_t *h_in = (uint8_t *)c.h_in.get(bin);
    uint8_t *h_meta = (uint8_t *)c.h_meta.get(meta_bytes);
    uint8_t *d_in = (uint8_t *)c.d_in.get(bin);
    uint8_t *d_out = (uint8_t *)c.d_out.get(bout);
    uint8_t *d_meta = (uint8_t *)c.d_meta.get(meta_bytes);
    uint64_t *m_in_off = (uint64_t *)h_meta, *m_out_off = m_in_off + n;
    uint32_t *m_in_len = (uint32_t *)(m_out_off + n), *m_out_cap = m_in_len + n;
    uint32_t *m_out_len = m_out_cap + n;
    int32_t *m_err = (int32_t *)(m_out_len + n);
    {
        uint64_t x = 0, y = 0;
        for (uint32_t k = 0; k < n; k++) {
            const uint32_t i = v.at(k);
            m_in_off[k] = x;
            m_out_off[k] = y;
            m_in_len[k] = a.in_len[i];
            m_out_cap[k] = a.out_cap[i];
            if (in_extent(a, i)) memcpy(h_in + x, a.in + a.in_off[i], in_extent(a, i));
            x += in_extent(a, i) ? in_extent(a, i) : 1u;
            y += a.out_cap[i];
        }
    }
    const size_t res_off = (uint8_t *)m_out_len - h_meta;
    check(hipMemcpyAsync(d_in, h_in, bin, hipMemcpyHostToDevice, c.stream), "hipMemcpyAsync");
    check(hipMemcpyAsync(d_meta, h_meta, res_off, hipMemcpyHostToDevice, c.stream), "hipMemcpyAsync");
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
    check(launch(a, b, c.stream), "kernel launch");
    check(hipMemcpyAsync(h_meta + res_off, d_meta + res_off, meta_bytes - res_off, hipMemcpyDeviceToHost,
                         c.stream),
          "hipMemcpyAsync");
    check(hipStreamSynchronize(c.stream), "hipStreamSynchronize");
    /* only the produced bytes come back: [lo, hi) of the packed outputs */
    uint64_t lo = ~0ull, hi = 0;
    for (uint32_t k = 0; k < n; k++) {
        const uint32_t i = v.at(k);
        a.out_len[i] = m_out_len[k];
        if (a.err) a.err[i] = m_err[k];
        if (!m_out_len[k]) continue;
        if (m_out_off[k] < lo) lo = m_out_off[k];
        if (m_out_off[k] + m_out_len[k] > hi) hi = m_out_off[k] + m_out_len[k];
    }
    if (hi > lo) {
        uint8_t *h_out = (uint8_t *)c.h_out.get(hi - lo);
        check(hipMemcpyAsync(h_out, d_out + lo, hi - lo, hipMemcpyDeviceToHost, c.stream), "hipMemcpyAsync");
        check(hipStreamSynchronize(c.stream), "hipStreamSynchronize");
        for (uint32_t k = 0; k < n; k++)
            if (m_out_len[k]) memcpy(a.out + a.out_off[v.at(k)], h_out + (m_out_off[k] - lo), m_out_len[k]);
    }
}

/* Registered arenas: no CPU byte copies.  Per chunk: descriptors up (pinned,
 * 48 B per value), the values into the packed device arena -- the DMA
 * engines copy runs of values that lie (nearly) back to back in the caller's
 * arena, the GPU gathers the rest from the mapped arena -- the routed
 * kernels, then the results into the caller's output slots -- decoded values
 * whose slots abut as DMA runs, streams by the GPU writing each one's
 * produced bytes -- and out_len / err come back with the descriptors.
 *
 * Chunks rotate over NSLOT slots, each with its own stream, buffers and
 * compress scratch, so chunk k+1's transfers run beside chunk k's kernels and
 * several chunks' compress launches run side by side: the one-lane-per-value
 * parse of a launch has a latency floor (~68 ms for 64 KiB values, DESIGN.md
 * §4.1) that mostly idles the GPU, so two or three overlapped launches cost
 * about one.  Compress batches of at least 192 MiB go in at least NSLOT
 * chunks (LZF_GPU_HOST_CHUNK_MB caps a chunk, default 4096) through the
 * routed generations whatever the chunk's count; decompress chunks hold
 * 256 MiB of output. */
void host_batch_mapped(Ctx &c, const HostArgs &a, const View &v, const uint8_t *in_map, uint8_t *out_map)
{
    make_slot_streams(c);
    /* per value: src_off, d_in_off, d_out_off, dst_off (u64), in_len, out_cap, out_len, err (u32) */
    const size_t mrec = 4 * sizeof(uint64_t) + 4 * sizeof(uint32_t);
    uint64_t total = 0;
    uint32_t max_len_all = 0;
    for (uint32_t k = 0; k < v.count; k++) {
        const uint32_t l = a.compress ? a.in_len[v.at(k)] : a.out_cap[v.at(k)];
        total += l;
        if (l > max_len_all) max_len_all = l;
    }
    uint32_t nchunks = 1;
    bool bulk = false;
    uint64_t chunk_bytes = 4096ull << 20;                  /* compress: the largest chunk's input */
    if (a.compress) {
        if (const char *e = getenv("LZF_GPU_HOST_CHUNK_MB")) chunk_bytes = (uint64_t)strtoull(e, nullptr, 10) << 20;
        if (chunk_bytes < (1u << 20)) chunk_bytes = 1u << 20;
        if (total >= (192ull << 20) && v.count >= NSLOT * 1024u) {
            nchunks = (uint32_t)((total + chunk_bytes - 1) / chunk_bytes);
            uint32_t nmin = NSLOT;
            if (const char *e = getenv("LZF_GPU_HOST_NCHUNKS")) nmin = (uint32_t)strtoul(e, nullptr, 10);
            if (nmin < 1u) nmin = 1u;
            if (nchunks < nmin) nchunks = nmin;
            bulk = true;
        }
    } else {
        uint64_t dchunk = 256ull << 20;
        if (const char *e = getenv("LZF_GPU_HOST_DCHUNK_MB")) dchunk = (uint64_t)strtoull(e, nullptr, 10) << 20;
        if (dchunk < (1u << 20)) dchunk = 1u << 20;
        nchunks = (uint32_t)((total + dchunk - 1) / dchunk);
    }
    if (nchunks > v.count) nchunks = v.count;
    if (nchunks < 1) nchunks = 1;
    /* equal chunks (measured: compress chunks shrinking toward the end, so
     * the last chunk's cand and scatter are short, were slower -- text64k
     * 202 -> 211 ms, json4k 62 -> 66 -- its cand squeezes between running
     * parses either way, and the parse's floor does not shrink with it) */
    std::vector<uint32_t> bound{0u};
    /* [lo, hi) as `parts` chunks of about equal bytes (value-aligned, none
     * empty), boundaries appended to `bound` */
    auto split_bytes = [&](uint32_t lo, uint32_t hi, uint32_t parts) {
        auto bytes_of = [&](uint32_t k) -> uint64_t { return a.compress ? a.in_len[v.at(k)] : a.out_cap[v.at(k)]; };
        uint64_t tot = 0;
        for (uint32_t k = lo; k < hi; k++) tot += bytes_of(k);
        if (parts > hi - lo) parts = hi - lo;
        uint64_t acc = 0;
        uint32_t k = lo;
        for (uint32_t p = 1; p < parts; p++) {
            const uint64_t target = tot * p / parts;
            while (k < hi && acc + bytes_of(k) <= target) acc += bytes_of(k++);
            if (k == bound.back() && k < hi) acc += bytes_of(k++);     /* never an empty chunk */
            if (k < hi) bound.push_back(k);
        }
        if (bound.back() != hi) bound.push_back(hi);
    };
    auto bytes_in = [&](uint32_t lo, uint32_t hi) {
        uint64_t t = 0;
        for (uint32_t k = lo; k < hi; k++) t += a.compress ? a.in_len[v.at(k)] : a.out_cap[v.at(k)];
        return t;
    };
    /* Tail mode (compress, values over 16 KiB): the first part of the batch
     * goes through the routed generations as one chunk, whose parse -- a
     * per-value chain of ~70 ms for 64 KiB values whatever the count --
     * starts as soon as that part is in; the rest is compressed by window64
     * (one wave per value, no such floor) in chunks as its input arrives,
     * beside that parse.  Without it every routed chunk's floor starts after
     * its own input, the last one after all of it.  The
     * routed part's share: LZF_GPU_HOST_TAIL (percent of the values, default
     * 70; 0 turns the mode off); window64 chunks: LZF_GPU_HOST_TAIL_CHUNKS
     * (1-4, default 1).  Both parts keep the chunk cap (LZF_GPU_HOST_CHUNK_MB,
     * default 4096): a routed share or window64 part past it is split into
     * chunks of at most that many input bytes, and chunks past the slots
     * reuse them in turn.  Registered text64k, 64 K values, compress GB/s
     * (profiles/r05/host_text64k_reg_tail*, tail_chunks/): four window
     * chunks by share: off 20.8, 30 % 21.6, 40 % 22.6, 50 % 23.9, 60 % 24.3,
     * 70 % 24.3, 80 % 23.0, 90 % 21.7; at 70 %, 1 / 2 / 3 / 4 chunks: 24.9 /
     * 24.4 / 24.4 / 24.3; one chunk at 60 / 80 %: 23.0 / 23.1. */
    uint32_t tail_from = v.count;
    if (bulk && max_len_all > 16384u && lzf_route_default()) {
        uint32_t pct = 70u;
        if (const char *e = getenv("LZF_GPU_HOST_TAIL")) pct = (uint32_t)strtoul(e, nullptr, 10);
        if (pct > 0u && pct < 100u) tail_from = (uint32_t)((uint64_t)v.count * pct / 100u);
    }
    if (tail_from < v.count) {
        uint32_t TAIL_CHUNKS = 1u;
        if (const char *e = getenv("LZF_GPU_HOST_TAIL_CHUNKS")) TAIL_CHUNKS = (uint32_t)strtoul(e, nullptr, 10);
        if (TAIL_CHUNKS < 1u) TAIL_CHUNKS = 1u;
        if (TAIL_CHUNKS > TAIL_MAX) TAIL_CHUNKS = TAIL_MAX;
        const uint64_t rb = bytes_in(0u, tail_from), tb = bytes_in(tail_from, v.count);
        split_bytes(0u, tail_from, (uint32_t)((rb + chunk_bytes - 1) / chunk_bytes));
        const uint32_t tcap = (uint32_t)((tb + chunk_bytes - 1) / chunk_bytes);
        split_bytes(tail_from, v.count, TAIL_CHUNKS > tcap ? TAIL_CHUNKS : tcap);
    } else {
        split_bytes(0u, v.count, nchunks);
    }
    const uint32_t min_len = a.compress ? 0u : 1u;

    auto drain = [&](Slot &sl) {
        if (!sl.busy) return;
        check(hipEventSynchronize(sl.done), "hipEventSynchronize");
        const uint32_t n = sl.count;
        const uint32_t *m_out_len = (const uint32_t *)((const uint64_t *)sl.h_meta.p + 4u * n) + 2u * n;
        const int32_t *m_err = (const int32_t *)(m_out_len + n);
        for (uint32_t k = 0; k < n; k++) {
            const uint32_t i = v.at(sl.first + k);
            a.out_len[i] = m_out_len[k];
            if (a.err) a.err[i] = m_err[k];
        }
        sl.busy = false;
    };
    struct Run {
        uint64_t host, dev, len;
    };
    std::vector<Run> iruns, oruns;
    std::vector<uint32_t> run_part;          /* the input part of each input run (cand parts) */
    std::vector<uint32_t> part_end;
    uint32_t round = 0;
    for (; round + 1 < bound.size(); round++) {
        const uint32_t k0 = bound[round], n = bound[round + 1] - k0;
        /* tail mode: every chunk its own slot while they last (the routed
         * chunk in slot 0 finishes last), so every chunk's input crosses the
         * bus as soon as the one before it is in (with two slots for four
         * chunks, the third waited for the first's kernel:
         * profiles/r05/tail_chunks/); past NSLOT_ALL chunks (a chunk cap far
         * below the batch) slots are reused in turn after draining */
        const uint32_t ns = tail_from == v.count ? NSLOT : NSLOT_ALL;
        const uint32_t si = round % ns;
        const uint32_t prev_si = round == 0u ? 0u : (round - 1u) % ns;
        Slot &sl = c.slot[si];
        drain(sl);
        uint8_t *h_meta = (uint8_t *)sl.h_meta.get((size_t)n * mrec);
        uint64_t *m_src = (uint64_t *)h_meta, *m_din = m_src + n, *m_dout = m_din + n, *m_dst = m_dout + n;
        uint32_t *m_in_len = (uint32_t *)(m_dst + n), *m_cap = m_in_len + n;
        /* Device offsets keep each value's host address mod 16 (whole 16-byte
         * moves).  Input runs: consecutive values at most 256 bytes apart in
         * the caller's arena are one DMA piece, gap bytes included (reads
         * only, inside the registered range).  Output runs (decode only):
         * slots that abut exactly, so a DMA piece writes only the call's own
         * slots. */
        iruns.clear();
        oruns.clear();
        /* Tail mode's routed chunk(s), inputs moved by DMA runs: the runs go
         * over the bus in LZF_GPU_HOST_CAND_PARTS parts (default 4) on the
         * context's input stream, and the table generation's kernel 1 runs
         * each part as it arrives, so the parse -- the per-value chain --
         * starts right after the last part instead of after a whole cand. */
        uint32_t nparts = 0;
        if (a.compress && bulk && k0 < tail_from && tail_from < v.count) {
            nparts = 4u;
            if (const char *e = getenv("LZF_GPU_HOST_CAND_PARTS")) nparts = (uint32_t)strtoul(e, nullptr, 10);
            if (nparts > 16u) nparts = 16u;
            if (nparts > n) nparts = n;
            if (nparts < 2u) nparts = 0u;
        }
        run_part.clear();
        uint32_t part_of_k = 0;
        uint64_t x = 0, y = 0;
        uint32_t max_len = 0;
        /* a decode chunk whose inputs' whole span is no larger than its
         * outputs goes H2D as that one span, gaps included: the bus's H2D
         * side idles while the D2H side carries the decoded bytes, and a GPU
         * gather's read requests would slow that D2H side */
        bool span = false;
        uint64_t slo = ~0ull, shi = 0;
        if (!a.compress) {
            uint64_t outb = 0;
            for (uint32_t k = 0; k < n; k++) {
                const uint32_t i = v.at(k0 + k);
                const uint64_t so = a.in_off[i], ext = in_extent(a, i);
                if (so < slo) slo = so;
                if (so + ext > shi) shi = so + ext;
                outb += a.out_cap[i];
            }
            span = n > 1u && shi - slo <= outb;
            if (span) {
                x = ((uintptr_t)in_map + slo) & 15u;
                iruns.push_back(Run{slo, x, shi - slo});
            }
        }
        for (uint32_t k = 0; k < n; k++) {
            const uint32_t i = v.at(k0 + k);
            const uint64_t so = a.in_off[i], ext = in_extent(a, i);
            if (span) {
                m_din[k] = iruns[0].dev + (so - slo);
            } else if (!iruns.empty() && so >= iruns.back().host + iruns.back().len &&
                       so - (iruns.back().host + iruns.back().len) <= 256u &&
                       !(nparts && (uint64_t)k * nparts / n != part_of_k)) {
                Run &r = iruns.back();
                m_din[k] = r.dev + (so - r.host);
                if (so + ext - r.host > r.len) r.len = so + ext - r.host;
            } else {
                x = ((x + 15u) & ~15ull) + (((uintptr_t)in_map + so) & 15u);
                iruns.push_back(Run{so, x, ext});
                m_din[k] = x;
                if (nparts) part_of_k = (uint32_t)((uint64_t)k * nparts / n);
                run_part.push_back(part_of_k);
            }
            if (m_din[k] + ext > x) x = m_din[k] + ext;           /* span: x ends at the span's end */
            const uint64_t oo = a.out_off[i];
            if (!a.compress && !oruns.empty() && oo == oruns.back().host + oruns.back().len) {
                Run &r = oruns.back();
                m_dout[k] = r.dev + r.len;
                r.len += a.out_cap[i];
            } else {
                y = ((y + 15u) & ~15ull) + (((uintptr_t)out_map + oo) & 15u);
                oruns.push_back(Run{oo, y, a.out_cap[i]});
                m_dout[k] = y;
            }
            y = m_dout[k] + a.out_cap[i];
            m_src[k] = so;
            m_dst[k] = oo;
            m_in_len[k] = a.in_len[i];
            m_cap[k] = a.out_cap[i];
            const uint32_t l = a.compress ? a.in_len[i] : a.out_cap[i];
            if (l > max_len) max_len = l;
        }
        uint8_t *d_in = (uint8_t *)sl.d_in.get(x + 16);
        uint8_t *d_out = (uint8_t *)sl.d_out.get(y + 16);
        uint8_t *d_meta = (uint8_t *)sl.d_meta.get((size_t)n * mrec);
        const size_t res_off = (uint8_t *)(m_cap + n) - h_meta;
        check(hipMemcpyAsync(d_meta, h_meta, res_off, hipMemcpyHostToDevice, sl.stream), "hipMemcpyAsync");
        const uint64_t *d_src = (const uint64_t *)d_meta, *d_din = d_src + n, *d_dout = d_din + n,
                       *d_dst = d_dout + n;
        const uint32_t *d_in_len = (const uint32_t *)(d_dst + n), *d_cap = d_in_len + n;
        uint32_t *d_out_len = (uint32_t *)(d_cap + n);
        const size_t few = 8u + n / 64u;
        /* the chunks' inputs cross the bus one chunk after the other (side by
         * side they would share the link and all arrive at the end): chunk
         * k's kernels then start when its own inputs are in */
        LzfParts parts{0u, nullptr, nullptr};
        if (nparts && iruns.size() > few) nparts = 0;       /* a gathered chunk arrives whole */
        if (nparts) {
            if (!c.in_stream) check(hipStreamCreateWithFlags(&c.in_stream, hipStreamNonBlocking), "hipStreamCreate");
            while (c.in_ev.size() < nparts) {
                hipEvent_t ev;
                check(hipEventCreateWithFlags(&ev, hipEventDisableTiming), "hipEventCreate");
                c.in_ev.push_back(ev);
            }
            if (round) check(hipStreamWaitEvent(c.in_stream, c.slot[prev_si].in_done, 0), "hipStreamWaitEvent");
            part_end.assign(nparts, 0u);
            for (uint32_t j = 0; j < nparts; j++) {
                part_end[j] = (uint32_t)((uint64_t)n * (j + 1u) / nparts);
                for (size_t r = 0; r < iruns.size(); r++)
                    if (run_part[r] == j && iruns[r].len)
                        check(hipMemcpyAsync(d_in + iruns[r].dev, a.in + iruns[r].host, iruns[r].len,
                                             hipMemcpyHostToDevice, c.in_stream),
                              "hipMemcpyAsync");
                check(hipEventRecord(c.in_ev[j], c.in_stream), "hipEventRecord");
            }
            parts = LzfParts{nparts, part_end.data(), c.in_ev.data()};
            /* the descriptors go up on the slot's stream; the kernels wait for the parts */
        } else {
        if (round) check(hipStreamWaitEvent(sl.stream, c.slot[prev_si].in_done, 0), "hipStreamWaitEvent");
        if (iruns.size() <= few) {
            for (const Run &r : iruns)
                if (r.len)
                    check(hipMemcpyAsync(d_in + r.dev, a.in + r.host, r.len, hipMemcpyHostToDevice, sl.stream),
                          "hipMemcpyAsync");
        } else {
            check(lzf_launch_move(in_map, d_src, d_in, d_din, d_in_len, min_len, n, sl.stream), "gather launch");
        }
        }
        check(hipEventRecord(sl.in_done, nparts ? c.in_stream : sl.stream), "hipEventRecord");
        LzfBatch b{};
        b.in = d_in;
        b.in_off = d_din;
        b.in_len = d_in_len;
        b.out = d_out;
        b.out_off = d_dout;
        b.out_cap = d_cap;
        b.out_len = d_out_len;
        b.err = (int32_t *)(d_out_len + n);
        b.count = n;
        b.max_len = max_len;
        const bool tail = k0 >= tail_from;
        check(tail   ? lzf_route_compress_window(b, sl.stream)
              : bulk ? lzf_route_compress_bulk(b, sl.stream, sl.scratch, nparts ? &parts : nullptr)
                     : launch(a, b, sl.stream),
              "kernel launch");
        /* outputs cross the bus in chunk order too: side by side, the chunks
         * in flight would share the link and finish together, leaving it idle
         * while the next ones gather and decode (not in tail mode: the
         * routed chunk finishes last) */
        if (round && CHAIN_OUT && tail_from == v.count)
            check(hipStreamWaitEvent(sl.stream, c.slot[prev_si].out_done, 0), "hipStreamWaitEvent");
        if (!a.compress && oruns.size() <= few) {
            /* a run carries whole slots: zero each slot past its decoded
             * length first, so no stale device bytes (an earlier chunk's or
             * batch's values) reach the caller's memory */
            check(lzf_launch_clear_tail(d_out, d_dout, d_out_len, d_cap, n, sl.stream), "clear launch");
            for (const Run &r : oruns)
                if (r.len)
                    check(hipMemcpyAsync(a.out + r.host, d_out + r.dev, r.len, hipMemcpyDeviceToHost, sl.stream),
                          "hipMemcpyAsync");
        } else {
            check(lzf_launch_move(d_out, d_dout, out_map, d_dst, d_out_len, 0u, n, sl.stream), "scatter launch");
        }
        check(hipEventRecord(sl.out_done, sl.stream), "hipEventRecord");
        check(hipMemcpyAsync(h_meta + res_off, d_meta + res_off, (size_t)n * mrec - res_off, hipMemcpyDeviceToHost,
                             sl.stream),
              "hipMemcpyAsync");
        check(hipEventRecord(sl.done, sl.stream), "hipEventRecord");
        sl.first = k0;
        sl.count = n;
        sl.busy = true;
    }
    for (uint32_t k = 0; k < NSLOT_ALL; k++) drain(c.slot[k]);
    if (c.in_stream) check(hipStreamSynchronize(c.in_stream), "hipStreamSynchronize");
}

/* the [lo, hi) byte ranges a sub-batch reads and writes in the caller's arenas */
void spans(const HostArgs &a, const View &v, uintptr_t &ilo, uintptr_t &ihi, uintptr_t &olo, uintptr_t &ohi)
{
    ilo = olo = UINTPTR_MAX;
    ihi = ohi = 0;
    for (uint32_t k = 0; k < v.count; k++) {
        const uint32_t i = v.at(k);
        const uintptr_t s = (uintptr_t)a.in + a.in_off[i], d = (uintptr_t)a.out + a.out_off[i];
        if (s < ilo) ilo = s;
        if (s + in_extent(a, i) > ihi) ihi = s + in_extent(a, i);
        if (d < olo) olo = d;
        if (d + a.out_cap[i] > ohi) ohi = d + a.out_cap[i];
    }
    if (ihi < ilo) ihi = ilo;
    if (ohi < olo) ohi = olo;
}

void host_batch(Ctx &c, const HostArgs &a, const View &v)
{
    DeviceGuard g(c.dev);
    uintptr_t ilo, ihi, olo, ohi;
    spans(a, v, ilo, ihi, olo, ohi);
    if (is_registered(ilo, ihi) && is_registered(olo, ohi)) {
        void *im = nullptr, *om = nullptr;
        /* device addresses of the arenas' bases (the ranges are mapped) */
        if (hipHostGetDevicePointer(&im, (void *)ilo, 0) == hipSuccess &&
            hipHostGetDevicePointer(&om, (void *)olo, 0) == hipSuccess) {
            host_batch_mapped(c, a, v, (const uint8_t *)im - (ilo - (uintptr_t)a.in),
                              (uint8_t *)om - (olo - (uintptr_t)a.out));
            return;
        }
        (void)hipGetLastError();
    }
    uint64_t sin = 0, sout = 0;
    for (uint32_t k = 0; k < v.count; k++) {
        const uint32_t i = v.at(k);
        sin += in_extent(a, i) ? in_extent(a, i) : 1u;
        sout += a.out_cap[i];
    }
    /* large batches whose outputs are not much bigger than their inputs go
     * through the chunked pipeline */
    const uint64_t chunk = 32ull << 20;
    if (sin >= 2 * chunk && sout <= 4 * sin)
        host_batch_staged(c, a, v, chunk, 4 * chunk);
    else
        host_batch_small(c, a, v);
}

/* a sub-batch on one context, failures as a return code (a host allocation
 * or thread-creation failure too: nothing may escape into the server) */
int host_run(Ctx &c, const HostArgs &a, const View &v)
{
    try {
        host_batch(c, a, v);
        return LZF_GPU_OK;
    } catch (const LzfFail &f) {
        c.quiesce();
        return f.code;
    } catch (...) {
        c.quiesce();
        return LZF_GPU_ENOMEM;
    }
}

/* ---- decoded sizes of host streams (the pre-pass of lzf_dsize.hip) -------- */

void host_dsize(Ctx &c, const uint8_t *in, const uint64_t *in_off, const uint32_t *in_len, uint32_t *out_size,
                int32_t *err, const View &v, uint32_t limit)
{
    DeviceGuard g(c.dev);
    const uint32_t n = v.count;
    uint64_t bin = 0;
    for (uint32_t k = 0; k < n; k++) bin += in_len[v.at(k)] ? in_len[v.at(k)] : 1u;
    const size_t mb = (size_t)n * (sizeof(uint64_t) + 3 * sizeof(uint32_t));
    uint8_t *h_in = (uint8_t *)c.h_in.get(bin), *h_meta = (uint8_t *)c.h_meta.get(mb);
    uint8_t *d_in = (uint8_t *)c.d_in.get(bin), *d_meta = (uint8_t *)c.d_meta.get(mb);
    uint64_t *m_off = (uint64_t *)h_meta;
    uint32_t *m_len = (uint32_t *)(m_off + n);
    uint64_t x = 0;
    for (uint32_t k = 0; k < n; k++) {
        const uint32_t i = v.at(k);
        const uint32_t e = in_len[i] ? in_len[i] : 1u;     /* a 0-length stream reads 1 byte */
        memcpy(h_in + x, in + in_off[i], e);
        m_off[k] = x;
        m_len[k] = in_len[i];
        x += e;
    }
    const size_t res = (size_t)n * (sizeof(uint64_t) + sizeof(uint32_t));
    check(hipMemcpyAsync(d_in, h_in, bin, hipMemcpyHostToDevice, c.stream), "hipMemcpyAsync");
    check(hipMemcpyAsync(d_meta, h_meta, res, hipMemcpyHostToDevice, c.stream), "hipMemcpyAsync");
    check(lzf_launch_dsize(d_in, (const uint64_t *)d_meta, (const uint32_t *)(d_meta + (size_t)n * sizeof(uint64_t)),
                           (uint32_t *)(d_meta + res), (int32_t *)(d_meta + res + (size_t)n * sizeof(uint32_t)), n,
                           limit, c.stream),
          "kernel launch");
    check(hipMemcpyAsync(h_meta + res, d_meta + res, mb - res, hipMemcpyDeviceToHost, c.stream), "hipMemcpyAsync");
    check(hipStreamSynchronize(c.stream), "hipStreamSynchronize");
    const uint32_t *r_size = (const uint32_t *)(h_meta + res);
    const int32_t *r_err = (const int32_t *)(r_size + n);
    for (uint32_t k = 0; k < n; k++) {
        out_size[v.at(k)] = r_size[k];
        err[v.at(k)] = r_err[k];
    }
}

/* ---- the per-device workers ---------------------------------------------- */

struct Worker {
    int dev = 0;
    int numa = -1;
    bool bound = false;
    bool ready = false;
    std::unique_ptr<Ctx> ctx;
    std::mutex mu;
    std::condition_variable cv;
    std::deque<std::function<void()>> q;
    std::thread th;

    explicit Worker(int d) : dev(d)
    {
        th = std::thread([this] { run(); });
        std::unique_lock<std::mutex> lk(mu);
        cv.wait(lk, [this] { return ready; });
    }
    void run()
    {
        cpu_set_t local;
        const int node = device_numa(dev, &local);
        const bool b = bind_to_node(node, local);
        (void)hipSetDevice(dev);
        std::unique_ptr<Ctx> c(new Ctx(dev, b));
        {
            std::lock_guard<std::mutex> lk(mu);
            numa = node;
            bound = b;
            ctx = std::move(c);
            ready = true;
        }
        cv.notify_all();
        for (;;) {
            std::function<void()> f;
            {
                std::unique_lock<std::mutex> lk(mu);
                cv.wait(lk, [this] { return !q.empty(); });
                f = std::move(q.front());
                q.pop_front();
            }
            f();
        }
    }
    void post(std::function<void()> f)
    {
        {
            std::lock_guard<std::mutex> lk(mu);
            q.push_back(std::move(f));
        }
        cv.notify_all();
    }
};

/* one worker per plan entry, made on first use and kept for the process's
 * life (its thread waits on its queue; process exit ends it).  Returns only
 * with every entry's worker made: when making one throws (a thread or memory
 * that could not be had), the vector keeps the workers made so far, the
 * exception reaches the caller (who returns LZF_GPU_ENOMEM), and the next
 * call goes on from there -- no caller ever sees a partial plan. */
std::mutex g_workers_mu;
std::vector<Worker *> g_workers;
std::vector<Worker *> &workers()
{
    std::mutex &mu = g_workers_mu;
    std::vector<Worker *> &w = g_workers;
    std::lock_guard<std::mutex> lk(mu);
    const std::vector<int> &dev = plan().dev;
    while (w.size() < dev.size()) {
        /* LZF_GPU_FORCE_WORKER_FAIL=<entry>: making that entry's worker
         * fails (tests of the partial-plan path) */
        const char *ff = getenv("LZF_GPU_FORCE_WORKER_FAIL");
        if (ff && *ff && (size_t)atoi(ff) == w.size()) throw std::bad_alloc();
        std::unique_ptr<Worker> x(new Worker(dev[w.size()]));
        w.push_back(x.get());
        x.release();
    }
    return w;
}

/* completion of the entries of one call */
struct Join {
    std::mutex mu;
    std::condition_variable cv;
    uint32_t left = 0;
    int rc = LZF_GPU_OK;
    void done(int r)
    {
        std::lock_guard<std::mutex> lk(mu);
        if (r != LZF_GPU_OK && rc == LZF_GPU_OK) rc = r;
        if (--left == 0) cv.notify_all();
    }
    int wait()
    {
        std::unique_lock<std::mutex> lk(mu);
        cv.wait(lk, [this] { return left == 0; });
        return rc;
    }
};

struct Spread {
    uint32_t values = 0;
    double ms = 0;
};
thread_local std::vector<Spread> g_spread;

/* Run job(ctx, view) for every plan entry's share of `count` values (value i
 * to entry i mod G) on the entries' workers, or on the calling thread when
 * there is one entry or one value. */
int dispatch(uint32_t count, const std::function<int(Ctx &, const View &)> &job)
{
    const Plan &P = plan();
    if (P.rc != LZF_GPU_OK) return P.rc;
    const uint32_t G = (uint32_t)P.dev.size();
    const bool block = lzf_host_split_policy() == 1;
    g_spread.assign(G, Spread{});
    if (G <= 1 || count == 1) {
        const auto t0 = std::chrono::steady_clock::now();
        int rc;
        try {
            rc = job(caller_ctx(), View{0, 1, count});
        } catch (const LzfFail &f) {
            rc = f.code;
        } catch (...) {
            rc = LZF_GPU_ENOMEM;
        }
        g_spread[0].values = count;
        g_spread[0].ms = std::chrono::duration<double, std::milli>(std::chrono::steady_clock::now() - t0).count();
        return rc;
    }
    std::vector<Worker *> *wp = nullptr;
    try {
        wp = &workers();
    } catch (...) {
        return LZF_GPU_ENOMEM;                     /* a worker thread could not be made */
    }
    std::vector<Worker *> &w = *wp;
    if (w.size() != G) return LZF_GPU_ENOMEM;
    Join j;
    j.left = G;
    for (uint32_t d = 0; d < G; d++) {
        View v;
        v.count = block ? lzf_host_split_block(count, G, d, &v.first) : lzf_host_split(count, G, d, &v.first, &v.stride);
        if (block) v.stride = 1u;
        g_spread[d].values = v.count;
        if (!v.count || !w[d]->ctx->ok) {
            j.done(v.count ? LZF_GPU_ENODEV : LZF_GPU_OK);
            continue;
        }
        Spread *sp = &g_spread[d];
        Ctx *c = w[d]->ctx.get();
        w[d]->post([&j, &job, c, v, sp] {
            const auto t0 = std::chrono::steady_clock::now();
            int rc;
            try {
                rc = job(*c, v);
            } catch (const LzfFail &f) {
                rc = f.code;
            } catch (...) {
                rc = LZF_GPU_ENOMEM;
            }
            sp->ms = std::chrono::duration<double, std::milli>(std::chrono::steady_clock::now() - t0).count();
            j.done(rc);
        });
    }
    return j.wait();
}

int host_batch_call(const HostArgs &a, uint32_t count)
{
    if (!count || !a.in || !a.in_off || !a.in_len || !a.out || !a.out_off || !a.out_cap || !a.out_len)
        return LZF_GPU_EARG;
    return dispatch(count, [&a](Ctx &c, const View &v) { return host_run(c, a, v); });
}

}  // namespace

extern "C" {

/* Single calls are batches of one, on the calling thread's context (the
 * plan's first device).  A failure of the device path (no usable gfx950, a
 * HIP error) is reported, never aborted on: lzf_compress returns 0, which the
 * caller already reads as "store the value plain" (src/query.c:393-397);
 * lzf_decompress returns 0 with errno EIO, an errno the reference codec never
 * sets (src/lzf.h:85-91 lists E2BIG and EINVAL). */
unsigned int lzf_compress(const void *const in_data, unsigned int in_len, void *out_data, unsigned int out_len)
{
    if (!in_len || !out_len) return 0;                    /* src/lzf_c.c:131 */
    if (!in_data || !out_data) return 0;
    uint64_t zero = 0;
    uint32_t res = 0;
    const HostArgs a{true, (const uint8_t *)in_data, &zero, &in_len, (uint8_t *)out_data, &zero, &out_len, &res,
                     nullptr};
    return host_batch_call(a, 1) == LZF_GPU_OK ? res : 0u;
}

unsigned int lzf_decompress(const void *const in_data, unsigned int in_len, void *out_data, unsigned int out_len)
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
    const HostArgs a{false, (const uint8_t *)in_data, &zero, &in_len, (uint8_t *)out_data, &zero, &out_len, &res,
                     &err};
    if (host_batch_call(a, 1) != LZF_GPU_OK) {
        errno = EIO;
        return 0;
    }
    if (!res) errno = err ? err : EINVAL;
    return res;
}

int lzf_host_compress_batch(const uint8_t *in, const uint64_t *in_off, const uint32_t *in_len, uint8_t *out,
                            const uint64_t *out_off, const uint32_t *out_cap, uint32_t *out_len, uint32_t count)
{
    return host_batch_call(HostArgs{true, in, in_off, in_len, out, out_off, out_cap, out_len, nullptr}, count);
}

int lzf_host_decompress_batch(const uint8_t *in, const uint64_t *in_off, const uint32_t *in_len, uint8_t *out,
                              const uint64_t *out_off, const uint32_t *out_cap, uint32_t *out_len, int32_t *err,
                              uint32_t count)
{
    if (!err) return LZF_GPU_EARG;
    return host_batch_call(HostArgs{false, in, in_off, in_len, out, out_off, out_cap, out_len, err}, count);
}

int lzf_host_decoded_size_batch(const uint8_t *in, const uint64_t *in_off, const uint32_t *in_len,
                                uint32_t *out_size, int32_t *err, uint32_t count, uint32_t out_limit)
{
    if (!count || !in || !in_off || !in_len || !out_size || !err) return LZF_GPU_EARG;
    return dispatch(count, [=](Ctx &c, const View &v) {
        try {
            host_dsize(c, in, in_off, in_len, out_size, err, v, out_limit);
            return LZF_GPU_OK;
        } catch (const LzfFail &f) {
            c.quiesce();
            return f.code;
        } catch (...) {
            c.quiesce();
            return LZF_GPU_ENOMEM;
        }
    });
}

int lzf_host_register(const void *ptr, uint64_t len)
{
    if (!ptr || !len) return LZF_GPU_EARG;
    const uintptr_t lo = (uintptr_t)ptr, hi = lo + len;
    const Plan &P = plan();
    if (P.rc != LZF_GPU_OK) return P.rc;
    /* the range is reserved as [lo, lo) while hipHostRegister runs outside
     * the lock (no batch span fits an empty range, and an overlapping or
     * second registration of it is refused), then entered whole */
    {
        std::lock_guard<std::mutex> lk(g_reg_mu);
        auto it = g_reg.upper_bound(lo);
        if (it != g_reg.end() && it->first < hi) return LZF_GPU_EARG;          /* overlaps a later range */
        if (it != g_reg.begin() && std::prev(it)->second > lo) return LZF_GPU_EARG;
        if (g_reg.count(lo)) return LZF_GPU_EARG;                               /* being registered */
        g_reg[lo] = lo;
    }
    int prev = -1;
    (void)hipGetDevice(&prev);
    hipError_t e = hipSetDevice(P.dev[0]);
    /* portable: registered once, pinned for every device */
    if (e == hipSuccess) e = hipHostRegister((void *)ptr, len, hipHostRegisterMapped | hipHostRegisterPortable);
    /* and mapped on each device of the plan: a batch's worker asks for the
     * arena's device address on its own device (host_batch), so the range is
     * refused here, whole, unless every plan device gives one -- for the
     * first and the last byte */
    if (e == hipSuccess) {
        const int rc = register_check_devices(P.dev, ptr, len);
        if (rc != LZF_GPU_OK) {
            (void)hipSetDevice(P.dev[0]);
            (void)hipHostUnregister((void *)ptr);
            if (prev >= 0) (void)hipSetDevice(prev);
            std::lock_guard<std::mutex> lk(g_reg_mu);
            g_reg.erase(lo);
            return rc;
        }
    }
    if (prev >= 0 && prev != P.dev[0]) (void)hipSetDevice(prev);
    std::lock_guard<std::mutex> lk(g_reg_mu);
    if (e != hipSuccess) {
        (void)hipGetLastError();
        g_reg.erase(lo);
        return code_of(e);
    }
    g_reg[lo] = hi;
    return LZF_GPU_OK;
}

int lzf_host_unregister(const void *ptr)
{
    {
        std::lock_guard<std::mutex> lk(g_reg_mu);
        auto it = g_reg.find((uintptr_t)ptr);
        if (it == g_reg.end() || it->second == it->first) return LZF_GPU_EARG;   /* unknown, or being registered */
        g_reg.erase(it);
    }
    return hipHostUnregister((void *)ptr) == hipSuccess ? LZF_GPU_OK : LZF_GPU_ELAUNCH;
}

int lzf_gpu_parse_device_list(const char *spec, int visible, int *dev, int max)
{
    if (!spec || !dev || max <= 0) return LZF_GPU_EARG;
    if (!strcmp(spec, "all")) {
        int n = 0;
        for (int d = 0; d < visible && n < max; d++) dev[n++] = d;
        return n > 0 ? n : LZF_GPU_ENODEV;
    }
    int n = 0;
    const char *s = spec;
    while (*s) {
        while (*s == ' ') s++;
        char *end;
        const long d = strtol(s, &end, 10);
        if (end == s || d < 0 || d >= visible || n >= max) return end == s || n >= max ? LZF_GPU_EARG : LZF_GPU_ENODEV;
        dev[n++] = (int)d;
        s = end;
        while (*s == ' ') s++;
        if (*s == ',') s++;
        else if (*s) return LZF_GPU_EARG;
    }
    return n > 0 ? n : LZF_GPU_EARG;
}

uint32_t lzf_host_split(uint32_t count, uint32_t groups, uint32_t g, uint32_t *first, uint32_t *stride)
{
    if (first) *first = g;
    if (stride) *stride = groups ? groups : 1u;
    if (!groups || g >= groups || g >= count) return 0;
    return (count - g + groups - 1u) / groups;
}

uint32_t lzf_host_split_block(uint32_t count, uint32_t groups, uint32_t g, uint32_t *first)
{
    if (!groups || g >= groups) {
        if (first) *first = 0;
        return 0;
    }
    const uint32_t lo = (uint32_t)((uint64_t)count * g / groups), hi = (uint32_t)((uint64_t)count * (g + 1) / groups);
    if (first) *first = lo;
    return hi - lo;
}

int lzf_host_split_policy(void)
{
    const char *e = getenv("LZF_GPU_SPLIT");
    return e && !strcmp(e, "block") ? 1 : 0;
}

int lzf_gpu_device_plan(int *device, int *numa_node, int *bound, int max)
{
    const Plan &P = plan();
    if (P.rc != LZF_GPU_OK) return P.rc;
    const int G = (int)P.dev.size();
    if (G > 1) {
        std::vector<Worker *> *wp = nullptr;
        try {
            wp = &workers();
        } catch (...) {
            return LZF_GPU_ENOMEM;
        }
        std::vector<Worker *> &w = *wp;
        for (int k = 0; k < G && k < max; k++) {
            if (device) device[k] = w[k]->dev;
            if (numa_node) numa_node[k] = w[k]->numa;
            if (bound) bound[k] = w[k]->bound ? 1 : 0;
        }
    } else if (max > 0) {
        cpu_set_t local;
        if (device) device[0] = P.dev[0];
        if (numa_node) numa_node[0] = device_numa(P.dev[0], &local);
        if (bound) bound[0] = 0;                           /* the calling thread is the caller's */
    }
    return G;
}

int lzf_host_last_spread(uint32_t *values, double *ms, int max)
{
    const int G = (int)g_spread.size();
    for (int k = 0; k < G && k < max; k++) {
        if (values) values[k] = g_spread[k].values;
        if (ms) ms[k] = g_spread[k].ms;
    }
    return G;
}

void lzf_gpu_release(void)
{
    lzf_scratch_release_all();
    if (t_caller) t_caller->release();
    if (plan().rc == LZF_GPU_OK && plan().dev.size() > 1) {
        /* only the workers already made (release makes none) */
        std::vector<Worker *> w;
        {
            std::lock_guard<std::mutex> lk(g_workers_mu);
            w = g_workers;
        }
        Join j;
        j.left = (uint32_t)w.size();
        for (Worker *x : w)
            x->post([&j, x] {
                x->ctx->release();
                j.done(LZF_GPU_OK);
            });
        j.wait();
    }
}

}  // extern "C"
