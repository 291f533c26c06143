// Read-bandwidth probe, variant 2 (not product code): the commit kernel's
// access pattern (2^20 rings of 16 KiB, each wave reads one ring's 8 KiB span
// from a random 16-B aligned start, wrapping; 64 lanes x 9 pieces of 16 B,
// depth-1 prefetch) with K dependent VALU instructions of "compute" placed
// after the next ring's loads are issued, as the commit kernel's walk + fold
// sit between its prefetch and its next staging.  Optionally each ring also
// reads a 64-B state row (as the kernel's per-group row).  Prints GB/s of
// the ring spans per K.  Answers: how much per-group compute (cycles of
// issue) can a wave do per 8 KiB window before the read rate drops?
// Usage: hipcc --offload-arch=gfx950 -O3 scripts/stream_probe2.hip -o /tmp/sp2 && /tmp/sp2
#include <hip/hip_runtime.h>
#include <stdio.h>
#include <stdint.h>

#define CK(x) do { hipError_t e_ = (x); if (e_ != hipSuccess) { printf("%s: %s\n", #x, hipGetErrorString(e_)); return 1; } } while (0)

constexpr uint32_t kRing = 16384, kSpan = 8192, kPPL = 9;
typedef uint32_t u32x4 __attribute__((ext_vector_type(4)));

__device__ __forceinline__ uint32_t start_of(uint32_t g) { return ((g * 2654435761u) >> 8) & (kRing - 16); }

template <int K, bool ROW, int DEPTH>
__global__ void __launch_bounds__(256) __attribute__((amdgpu_waves_per_eu(2)))
probe(const uint8_t *ring, const uint4 *rows, uint32_t G, uint32_t *out)
{
    const uint32_t lane = threadIdx.x & 63, wv = threadIdx.x >> 6;
    const uint32_t gstride = gridDim.x * 4;
    uint32_t acc = lane;
    u32x4 bufs[DEPTH][kPPL];
    uint4 row = {};
    auto issue = [&](u32x4 (&buf)[kPPL], uint32_t g) {
        const uint32_t gc = g < G ? g : G - 1;
        const __amdgpu_buffer_rsrc_t rs = __builtin_amdgcn_make_buffer_rsrc(
            const_cast<uint8_t *>(ring + (uint64_t)gc * kRing), (short)0, g < G ? (int)kRing : 0, 0x00020000);
        const uint32_t s = start_of(gc);
#pragma unroll
        for (int j = 0; j < (int)kPPL; ++j) {
            const uint32_t v = 16u * lane + 1024u * j;
            const uint32_t off = v < kSpan + 16 ? (s + v) & (kRing - 1) : 0xFFFFFFF0u;
            buf[j] = __builtin_amdgcn_raw_buffer_load_b128(rs, off, 0, 2);
        }
        if (ROW) row = rows[(uint64_t)gc * 4 + (lane & 3)];
    };
    uint32_t g = blockIdx.x * 4 + wv;
#pragma unroll
    for (int d = 0; d < DEPTH; ++d) issue(bufs[d], g + d * gstride);
    for (; g < G; g += DEPTH * gstride) {
#pragma unroll
        for (int d = 0; d < DEPTH; ++d) {
#pragma unroll
            for (int j = 0; j < (int)kPPL; ++j) acc ^= bufs[d][j].x ^ bufs[d][j].y ^ bufs[d][j].z ^ bufs[d][j].w;
            if (ROW) acc ^= row.x;
            asm volatile("" : "+v"(acc));
            issue(bufs[d], g + (d + DEPTH) * gstride);
            uint32_t x = acc;
            for (int k = 0; k < K; ++k) asm volatile("v_mad_u32_u24 %0, %0, 3, 1" : "+v"(x));
            acc ^= x & 1u;
        }
    }
    if (acc == 0x12345678u) out[0] = acc;
}

template <int K, bool ROW, int DEPTH>
static int run(const uint8_t *d, const uint4 *rows, uint32_t G, uint32_t *o, int wpc)
{
    hipEvent_t a, b;
    CK(hipEventCreate(&a)); CK(hipEventCreate(&b));
    float sum = 0.f;
    const int R = 10, grid = 256 * wpc / 4;
    for (int r = 0; r < R + 2; ++r) {
        CK(hipEventRecord(a));
        hipLaunchKernelGGL((probe<K, ROW, DEPTH>), dim3(grid), dim3(256), 0, 0, d, rows, G, o);
        CK(hipEventRecord(b));
        CK(hipEventSynchronize(b));
        float ms;
        CK(hipEventElapsedTime(&ms, a, b));
        if (r >= 2) sum += ms;
    }
    const double bytes = (double)G * (kSpan + 16);
    printf("waves/CU %2d depth %d K=%5d row=%d  avg %.4f ms  %.0f GB/s\n", wpc, DEPTH, K, ROW ? 1 : 0, sum / R,
           bytes / (sum / R * 1e6));
    return 0;
}

int main()
{
    const uint32_t G = 1u << 20;
    uint8_t *d;
    uint4 *rows;
    uint32_t *o;
    CK(hipMalloc(&d, (size_t)G * kRing));
    CK(hipMalloc(&rows, (size_t)G * 64));
    CK(hipMalloc(&o, 64));
    CK(hipMemset(d, 1, (size_t)G * kRing));
    CK(hipMemset(rows, 2, (size_t)G * 64));
    run<0, false, 1>(d, rows, G, o, 16);
    run<500, false, 1>(d, rows, G, o, 16);
    run<500, true, 1>(d, rows, G, o, 16);
    run<0, false, 1>(d, rows, G, o, 12);
    run<500, false, 1>(d, rows, G, o, 12);
    run<0, false, 2>(d, rows, G, o, 12);
    run<500, false, 2>(d, rows, G, o, 12);
    run<1000, false, 2>(d, rows, G, o, 12);
    run<0, false, 2>(d, rows, G, o, 8);
    run<500, false, 2>(d, rows, G, o, 8);
    run<1000, false, 2>(d, rows, G, o, 8);
    run<500, false, 1>(d, rows, G, o, 20);
    run<500, false, 1>(d, rows, G, o, 24);
    run<1000, false, 1>(d, rows, G, o, 24);
    run<500, false, 2>(d, rows, G, o, 16);
    CK(hipFree(d));
    CK(hipFree(rows));
    return 0;
}
