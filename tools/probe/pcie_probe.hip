// pcie_probe.hip -- what the host-memory batch path can get from PCIe on
// this box: hipHostRegister cost, hipMemcpyAsync from registered caller
// memory (each direction and both at once), and kernels that read / write
// mapped host memory directly (one workgroup per value, 16-byte accesses).
// Prints one JSON line.  usage: pcie_probe [MiB] [value_bytes]
#include <hip/hip_runtime.h>
#include <chrono>
#include <stdio.h>
#include <stdlib.h>
#include <string.h>

#define CK(x) do { hipError_t e_ = (x); if (e_ != hipSuccess) { \
    fprintf(stderr, "%s: %s\n", #x, hipGetErrorString(e_)); exit(1); } } while (0)

static double now() {
    return std::chrono::duration<double>(std::chrono::steady_clock::now().time_since_epoch()).count();
}

// value j: n bytes from src + j*n to dst + j*n (16-byte aligned)
__global__ __launch_bounds__(256) void copy_values(const uint4 *__restrict__ src, uint4 *__restrict__ dst, uint32_t n16)
{
    const uint64_t base = (uint64_t)blockIdx.x * n16;
    for (uint32_t k = threadIdx.x; k < n16; k += 4 * 256) {
        uint4 a = src[base + k];
        uint4 b = k + 256 < n16 ? src[base + k + 256] : uint4{};
        uint4 c = k + 512 < n16 ? src[base + k + 512] : uint4{};
        uint4 d = k + 768 < n16 ? src[base + k + 768] : uint4{};
        dst[base + k] = a;
        if (k + 256 < n16) dst[base + k + 256] = b;
        if (k + 512 < n16) dst[base + k + 512] = c;
        if (k + 768 < n16) dst[base + k + 768] = d;
    }
}

int main(int argc, char **argv)
{
    const size_t mib = argc > 1 ? strtoull(argv[1], 0, 10) : 1024;
    const uint32_t n = argc > 2 ? (uint32_t)strtoul(argv[2], 0, 10) : 65536;
    const size_t bytes = mib << 20;
    const uint32_t count = (uint32_t)(bytes / n);
    uint8_t *h = (uint8_t *)aligned_alloc(4096, bytes), *h2 = (uint8_t *)aligned_alloc(4096, bytes);
    memset(h, 1, bytes);
    memset(h2, 2, bytes);
    uint8_t *d, *d2;
    CK(hipMalloc(&d, bytes));
    CK(hipMalloc(&d2, bytes));
    hipStream_t s1, s2;
    CK(hipStreamCreateWithFlags(&s1, hipStreamNonBlocking));
    CK(hipStreamCreateWithFlags(&s2, hipStreamNonBlocking));
    double t0 = now();
    CK(hipHostRegister(h, bytes, hipHostRegisterMapped | hipHostRegisterPortable));
    double t_reg = now() - t0;
    CK(hipHostRegister(h2, bytes, hipHostRegisterMapped | hipHostRegisterPortable));
    void *hm, *hm2;
    CK(hipHostGetDevicePointer(&hm, h, 0));
    CK(hipHostGetDevicePointer(&hm2, h2, 0));
    auto rate = [&](auto f) {
        double best = 1e9;
        for (int r = 0; r < 4; r++) {
            CK(hipDeviceSynchronize());
            double a = now();
            f();
            CK(hipDeviceSynchronize());
            double t = now() - a;
            if (r && t < best) best = t;
        }
        return bytes / best / 1e9;
    };
    double h2d = rate([&] { CK(hipMemcpyAsync(d, h, bytes, hipMemcpyHostToDevice, s1)); });
    double d2h = rate([&] { CK(hipMemcpyAsync(h2, d, bytes, hipMemcpyDeviceToHost, s1)); });
    double duplex = rate([&] {
        CK(hipMemcpyAsync(d, h, bytes, hipMemcpyHostToDevice, s1));
        CK(hipMemcpyAsync(h2, d2, bytes, hipMemcpyDeviceToHost, s2));
    });
    // per-value copies (one hipMemcpyAsync per value): the cost of many small DMA calls
    double h2d_per = rate([&] {
        for (uint32_t j = 0; j < count; j++)
            CK(hipMemcpyAsync(d + (size_t)j * n, h + (size_t)j * n, n, hipMemcpyHostToDevice, s1));
    });
    const uint32_t n16 = n / 16;
    double zc_read = rate([&] { copy_values<<<count, 256, 0, s1>>>((const uint4 *)hm, (uint4 *)d, n16); });
    double zc_write = rate([&] { copy_values<<<count, 256, 0, s1>>>((const uint4 *)d, (uint4 *)hm2, n16); });
    double zc_duplex = rate([&] {
        copy_values<<<count, 256, 0, s1>>>((const uint4 *)hm, (uint4 *)d, n16);
        copy_values<<<count, 256, 0, s2>>>((const uint4 *)d2, (uint4 *)hm2, n16);
    });
    CK(hipDeviceSynchronize());
    bool ok = true;
    for (size_t i = 0; i < bytes; i += 4093) ok &= h2[i] == 1 || h2[i] == 2;
    t0 = now();
    CK(hipHostUnregister(h));
    double t_unreg = now() - t0;
    CK(hipHostUnregister(h2));
    printf("{\"MiB\": %zu, \"value_bytes\": %u, \"register_s\": %.4f, \"register_GBps\": %.1f, \"unregister_s\": %.4f, "
           "\"memcpy_h2d_GBps\": %.1f, \"memcpy_d2h_GBps\": %.1f, \"memcpy_duplex_GBps\": %.1f, "
           "\"memcpy_h2d_per_value_GBps\": %.2f, \"kernel_read_mapped_GBps\": %.1f, \"kernel_write_mapped_GBps\": %.1f, "
           "\"kernel_duplex_GBps\": %.1f, \"ok\": %s}\n",
           mib, n, t_reg, bytes / t_reg / 1e9, t_unreg, h2d, d2h, duplex, h2d_per, zc_read, zc_write, zc_duplex,
           ok ? "true" : "false");
    return 0;
}
