// Write-bandwidth probe for the append kernel's access pattern (not product
// code): 2^20 rings of 16 KiB, each wave appends 64 entries of 128 B at a
// random 16-B aligned start (wrapping), as log_append_entry writes them.
// log_append_entry never writes sender@27, bytes 41..47 or the 14 bytes past
// a command of 64 B (114..127), so the product reads each span before it
// writes it back in 16-B pieces.  Cases:
//   full16   16-B stores of every byte (no read: the bound without the span read)
//   rmw16    16-B loads of the span, then 16-B stores (the product's traffic)
//   masked   16-B stores of the pieces the reference writes whole, dword /
//            short / byte stores of the written bytes of the other pieces
//   rmwlds   the span read straight into LDS (buffer_load ... lds, 16 B per
//            lane, as append_kernel reads it), then LDS -> 16-B stores
//   rmwlds12 the same with append_kernel's LDS footprint (13.3 KB per wave:
//            3 blocks, 12 waves per CU)
// Usage: hipcc --offload-arch=gfx950 -O3 scripts/write_probe.hip -o /tmp/wp && /tmp/wp
#include <hip/hip_runtime.h>
#include <stdio.h>
#include <stdint.h>

#define CK(x) do { hipError_t e_ = (x); if (e_ != hipSuccess) { printf("%s: %s\n", #x, hipGetErrorString(e_)); return 1; } } while (0)

constexpr uint32_t kRing = 16384, kSpan = 8192;

__device__ __forceinline__ uint32_t start_of(uint32_t g) { return ((g * 2654435761u) >> 8) & (kRing - 16); }

template <int MODE>
__global__ void __launch_bounds__(256) __attribute__((amdgpu_waves_per_eu(4)))
probe(uint8_t *ring, uint32_t G, uint32_t salt)
{
    const uint32_t lane = threadIdx.x & 63, wv = threadIdx.x >> 6;
    const uint32_t gstride = gridDim.x * 4;
    extern __shared__ __attribute__((aligned(16))) uint4 s_dyn[];   // 4 waves x (8 KiB, or 13 KB for rmwlds12)
    uint4 *s_img_w = s_dyn + wv * ((MODE == 4 ? 13312u : kSpan) / 16u);
    for (uint32_t g = blockIdx.x * 4 + wv; g < G; g += gstride) {
        uint8_t *r = ring + (uint64_t)g * kRing;
        const uint32_t s = start_of(g);
        if (MODE >= 3) {
            const __amdgpu_buffer_rsrc_t rs = __builtin_amdgcn_make_buffer_rsrc(r, (short)0, (int)kRing, 0x00020000);
#pragma unroll
            for (int j = 0; j < 8; ++j)
                __builtin_amdgcn_raw_ptr_buffer_load_lds(rs, s_img_w + 64 * j, 16, (s + 16u * lane + 1024u * j) & (kRing - 1), 0, 0, 0);
            __builtin_amdgcn_s_waitcnt(0);
            asm volatile("" ::: "memory");
#pragma unroll
            for (int j = 0; j < 8; ++j) {
                uint4 x = s_img_w[64 * j + lane];
                x.x ^= salt;
                *reinterpret_cast<uint4 *>(r + ((s + 16u * lane + 1024u * j) & (kRing - 1))) = x;
            }
            asm volatile("" ::: "memory");
            continue;
        }
        uint4 v[8];
        if (MODE == 1) {
#pragma unroll
            for (int j = 0; j < 8; ++j) v[j] = *reinterpret_cast<const uint4 *>(r + ((s + 16u * lane + 1024u * j) & (kRing - 1)));
        }
#pragma unroll
        for (int j = 0; j < 8; ++j) {
            const uint32_t w = 16u * lane + 1024u * j;          // span offset (entry-relative: w & 127)
            const uint32_t off = (s + w) & (kRing - 1);
            uint4 d = make_uint4(w ^ salt, g, w + salt, g ^ salt);
            if (MODE == 1) d = make_uint4(v[j].x ^ salt, v[j].y, v[j].z, v[j].w);
            uint8_t *p = r + off;
            if (MODE != 2) {
                *reinterpret_cast<uint4 *>(p) = d;
            } else {
                const uint32_t pc = (w & 127u) >> 4;               // piece of the entry
                if (pc == 0 || (pc >= 3 && pc <= 6)) {
                    *reinterpret_cast<uint4 *>(p) = d;
                } else if (pc == 1) {                              // 16..26, 28..31 (sender@27 kept)
                    *reinterpret_cast<uint2 *>(p) = make_uint2(d.x, d.y);
                    *reinterpret_cast<uint16_t *>(p + 8) = (uint16_t)d.z;
                    p[10] = (uint8_t)(d.z >> 16);
                    *reinterpret_cast<uint32_t *>(p + 12) = d.w;
                } else if (pc == 2) {                              // 32..40 (41..47 kept)
                    *reinterpret_cast<uint2 *>(p) = make_uint2(d.x, d.y);
                    p[8] = (uint8_t)d.z;
                } else {                                           // 112..113 (114..127 kept)
                    *reinterpret_cast<uint16_t *>(p) = (uint16_t)d.x;
                }
            }
        }
    }
}

template <int MODE>
static int run(const char *name, uint8_t *d, uint32_t G, int grid)
{
    hipEvent_t a, b;
    CK(hipEventCreate(&a)); CK(hipEventCreate(&b));
    float best = 1e9f, sum = 0.f;
    const int R = 10;
    for (int i = 0; i < R + 2; ++i) {
        CK(hipEventRecord(a));
        const size_t lds = MODE == 4 ? 4 * 13312 : MODE == 3 ? 4 * kSpan : 0;
        hipLaunchKernelGGL(probe<MODE>, dim3(grid), dim3(256), lds, 0, d, G, (uint32_t)i);
        CK(hipEventRecord(b));
        CK(hipEventSynchronize(b));
        float ms;
        CK(hipEventElapsedTime(&ms, a, b));
        if (i >= 2) { sum += ms; if (ms < best) best = ms; }
    }
    const double wr = (double)G * kSpan;
    printf("%-8s best %.3f ms  mean %.3f ms  span bytes %.2f GB -> %.0f GB/s (best)\n", name, best, sum / R, wr / 1e9,
           wr / best / 1e6);
    return 0;
}

int main()
{
    const uint32_t G = 1u << 20;
    uint8_t *d;
    CK(hipMalloc(&d, (size_t)G * kRing));
    CK(hipMemset(d, 0, (size_t)G * kRing));
    int dev, ncu;
    CK(hipGetDevice(&dev));
    CK(hipDeviceGetAttribute(&ncu, hipDeviceAttributeMultiprocessorCount, dev));
    const int grid = ncu * 8;
    for (int rep = 0; rep < 2; ++rep) {
        if (run<0>("full16", d, G, grid)) return 1;
        if (run<1>("rmw16", d, G, grid)) return 1;
        if (run<2>("masked", d, G, grid)) return 1;
        if (run<3>("rmwlds", d, G, grid)) return 1;
        if (run<4>("rmwlds12", d, G, grid)) return 1;
    }
    CK(hipFree(d));
    return 0;
}
