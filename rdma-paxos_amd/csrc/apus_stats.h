// Per-block partial statistics shared by the kernels of libapus_gpu.
// Each block writes NSTAT values to partials[blockIdx.x * NSTAT + k]; one
// finalize launch folds them into ctx->stats (sum or min) — no contended
// atomics inside the streaming kernels.
#pragma once

#include <hip/hip_runtime.h>
#include <stdint.h>

namespace apus {

// MINMASK bit k: statistic k is a minimum (else a sum).  SC1: the row is
// stored write-through (sc1), for a reader in another block of the same
// launch (quorum_tail_kernel's last arriving block).
template <int NSTAT, uint32_t MINMASK = 0u, bool SC1 = false>
__device__ __forceinline__ void block_partials(uint64_t *partials, const uint64_t (&v)[NSTAT])
{
    __shared__ uint64_t red[16][NSTAT];
    const uint32_t lane = threadIdx.x & 63, wv = threadIdx.x >> 6, nw = (blockDim.x + 63) >> 6;
    uint64_t x[NSTAT];
#pragma unroll
    for (int k = 0; k < NSTAT; ++k) {
        uint64_t t = v[k];
        const bool MIN = (MINMASK >> k) & 1u;
#pragma unroll
        for (int d = 32; d >= 1; d >>= 1) {
            const uint64_t y = __shfl_xor(t, d);
            t = MIN ? (y < t ? y : t) : t + y;
        }
        x[k] = t;
    }
    if (lane == 0)
#pragma unroll
        for (int k = 0; k < NSTAT; ++k) red[wv][k] = x[k];
    __syncthreads();
    if (threadIdx.x < (uint32_t)NSTAT) {
        const bool MIN = (MINMASK >> threadIdx.x) & 1u;
        uint64_t s = MIN ? ~0ull : 0ull;
        for (uint32_t w = 0; w < nw; ++w) {
            const uint64_t y = red[w][threadIdx.x];
            s = MIN ? (y < s ? y : s) : s + y;
        }
        uint64_t *dst = &partials[(uint64_t)blockIdx.x * NSTAT + threadIdx.x];
        if (SC1) __hip_atomic_store(dst, s, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
        else *dst = s;
    }
}

// launched from apus_commit.hip; map: statistic k -> stats[(map >> 8k) & 0xFF],
// min_mask bit k: statistic k is folded by minimum (else summed)
hipError_t launch_stats_finalize(const uint64_t *partials, uint32_t nblk, uint32_t nstat,
                                 uint64_t *stats, uint64_t map, uint32_t min_mask, hipStream_t s,
                                 uint32_t *reset = nullptr);

}  // namespace apus
