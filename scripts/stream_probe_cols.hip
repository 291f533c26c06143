// Read-bandwidth probe (not product code): the commit tail's inputs at the
// 64M-group point (C4 on one GPU, R = 5) as the batch lays them out -- eight
// separate columns per group: the 64-B state row, remote_end and
// apply_offsets (40 B each), lr_step and fail_count (5 B each), self_idx and
// prev_head (1 B each), abs_base (8 B): 164 B per group -- against the same
// bytes as ONE array.  Kernels, each timed over REPS launches:
//   cols_lane   lane per group, every column element loaded (the tail's form)
//   cols_wave   per wave, each column's 64-group chunk read as 16-B pieces
//               (the LDS-staged form's loads, into registers)
//   one_stream  the single array, 16-B pieces, grid-stride
//   lane_st     cols_lane + the tail's four output streams (8 + 8 + 1 + 8 B
//               per group)
//   lane_st_cmp lane_st + arithmetic of the median's and pruning's shape
//               (circular distances, a rank selection over the R offsets)
//   lane_st_Nout lane_st with the first N output streams only (3: without the
//               1-B column; 2, 1: fewer 8-B columns)
//   lane_st_row the four outputs as ONE 32-B row per group (one write stream)
// Prints GB/s per kernel (bytes = 164 x G).  Answers: do eight column streams
// read slower than one stream of the same bytes, whatever the loads' form?
// Usage: hipcc --offload-arch=gfx950 -O3 scripts/stream_probe_cols.hip -o /tmp/spc && /tmp/spc
#include <hip/hip_runtime.h>
#include <stdio.h>
#include <stdint.h>

#define CK(x) do { hipError_t e_ = (x); if (e_ != hipSuccess) { printf("%s: %s\n", #x, hipGetErrorString(e_)); return 1; } } while (0)

constexpr int R = 5;
constexpr uint64_t kPerGroup = 64 + 8 * R + 8 * R + R + R + 1 + 1 + 8;   // 164

struct Cols {
    const uint4 *state;          // 64 B per group
    const uint64_t *rend, *ap;   // R per group
    const uint8_t *step, *fail;  // R per group
    const uint8_t *self, *prev;  // 1 per group
    const uint64_t *base;        // 1 per group
};

__global__ void __launch_bounds__(256) cols_lane(Cols c, uint64_t G, uint32_t *out)
{
    uint64_t acc = 0;
    for (uint64_t g = (uint64_t)blockIdx.x * 256 + threadIdx.x; g < G; g += (uint64_t)gridDim.x * 256) {
        uint4 s[4];
        for (int k = 0; k < 4; ++k) s[k] = c.state[4 * g + k];
        uint64_t v = 0;
        for (int i = 0; i < R; ++i) v += c.rend[R * g + i] ^ c.ap[R * g + i] ^ c.step[R * g + i] ^ c.fail[R * g + i];
        v += c.self[g] + c.prev[g] + c.base[g];
        for (int k = 0; k < 4; ++k) v += s[k].x ^ s[k].y ^ s[k].z ^ s[k].w;
        acc += v;
    }
    if (acc == 0x123456789ull) out[0] = 1;
}

struct Outs {
    uint64_t *med, *nh, *mn;
    uint8_t *ah;
    uint4 *row;   // lane_st_row: one 32-B row per group (median, new_head, min_apply, append_head)
};

__device__ __forceinline__ uint64_t cdist(uint64_t end, uint64_t len, uint64_t o)
{
    if (end == len) return 0;
    return end >= o ? end - o : len - (o - end);
}

template <bool CMP, int NOUT = 4>
__global__ void __launch_bounds__(256) lane_st(Cols c, Outs o, uint64_t G)
{
    for (uint64_t g = (uint64_t)blockIdx.x * 256 + threadIdx.x; g < G; g += (uint64_t)gridDim.x * 256) {
        uint4 s[4];
        for (int k = 0; k < 4; ++k) s[k] = c.state[4 * g + k];
        uint64_t re[R], ap[R];
        uint32_t st[R], fl[R];
        for (int i = 0; i < R; ++i) {
            re[i] = c.rend[R * g + i];
            ap[i] = c.ap[R * g + i];
            st[i] = c.step[R * g + i];
            fl[i] = c.fail[R * g + i];
        }
        const uint64_t self = c.self[g], prev = c.prev[g], base = c.base[g];
        const uint64_t commit = ((uint64_t)s[1].y << 32) | s[1].x, end = ((uint64_t)s[1].w << 32) | s[1].z;
        const uint64_t len = ((uint64_t)s[2].w << 32) | s[2].z, head = ((uint64_t)s[0].y << 32) | s[0].x;
        uint64_t med = commit ^ end ^ len ^ self ^ prev ^ base, mn = head;
        for (int i = 0; i < R; ++i) med += re[i] ^ ap[i] ^ st[i] ^ fl[i];
        if (CMP) {
            // the median's shape: R circular-distance tests, a rank selection
            // over R keys; pruning's: R circular minima
            uint64_t off[R];
            int cnt = 0;
            for (int i = 0; i < R; ++i) {
                off[i] = (i == (int)self) ? end : (st[i] == 5 && fl[i] < 3 ? re[i] : commit);
                cnt += cdist(end, len, off[i]) < cdist(end, len, commit) ? 1 : 0;
            }
            const uint32_t want = (uint32_t)(R - 1) / 2;
            for (int i = 0; i < R; ++i) {
                uint32_t r = 0;
                for (int k = 0; k < R; ++k)
                    if (k != i) r += (off[k] < off[i] || (off[k] == off[i] && k < i)) ? 1u : 0u;
                if (r == want) med = off[i] + cnt;
            }
            for (int i = 0; i < R; ++i)
                if (cdist(end, len, ap[i]) < cdist(end, len, mn)) mn = ap[i];
        }
        if (NOUT == 0) {
            const uint64_t nh = mn + 1, ah = mn > head;
            o.row[2 * g] = make_uint4((uint32_t)med, (uint32_t)(med >> 32), (uint32_t)nh, (uint32_t)(nh >> 32));
            o.row[2 * g + 1] = make_uint4((uint32_t)mn, (uint32_t)(mn >> 32), (uint32_t)ah, 0);
            continue;
        }
        o.med[g] = med;
        if (NOUT >= 2) o.nh[g] = mn + 1;
        if (NOUT >= 3) o.mn[g] = mn;
        if (NOUT >= 4) o.ah[g] = (uint8_t)(mn > head);
    }
}

// state rows whose end != len, so the circular distances take their full path
__global__ void init_state(uint4 *st, uint64_t G)
{
    for (uint64_t g = (uint64_t)blockIdx.x * 256 + threadIdx.x; g < G; g += (uint64_t)gridDim.x * 256) {
        st[4 * g + 0] = make_uint4((uint32_t)(g * 7) & 0x1FFF, 0, 1, 0);
        st[4 * g + 1] = make_uint4((uint32_t)(g % 9000), 0, (uint32_t)((g * 13) % 9000), 0);
        st[4 * g + 2] = make_uint4(0, 0, 9000, 0);
        st[4 * g + 3] = make_uint4(0, 0, 0, 0);
    }
}

__device__ __forceinline__ uint64_t chunk(const void *col, uint64_t g0, uint32_t elt, uint32_t lane)
{
    const uint4 *p = reinterpret_cast<const uint4 *>(static_cast<const uint8_t *>(col) + g0 * elt);
    const uint32_t np = (64u * elt) >> 4;
    uint64_t v = 0;
    for (uint32_t k = lane; k < np; k += 64) {
        const uint4 x = p[k];
        v += x.x ^ x.y ^ x.z ^ x.w;
    }
    return v;
}

__global__ void __launch_bounds__(256) cols_wave(Cols c, uint64_t G, uint32_t *out)
{
    const uint32_t lane = threadIdx.x & 63, wv = threadIdx.x >> 6;
    uint64_t acc = 0;
    for (uint64_t ch = (uint64_t)blockIdx.x * 4 + wv; ch * 64 + 64 <= G; ch += (uint64_t)gridDim.x * 4) {
        const uint64_t g0 = ch * 64;
        acc += chunk(c.state, g0, 64, lane) + chunk(c.rend, g0, 8 * R, lane) + chunk(c.ap, g0, 8 * R, lane) +
               chunk(c.step, g0, R, lane) + chunk(c.fail, g0, R, lane) + chunk(c.self, g0, 1, lane) +
               chunk(c.prev, g0, 1, lane) + chunk(c.base, g0, 8, lane);
    }
    if (acc == 0x123456789ull) out[0] = 1;
}

__global__ void __launch_bounds__(256) one_stream(const uint4 *a, uint64_t n16, uint32_t *out)
{
    uint64_t acc = 0;
    for (uint64_t i = (uint64_t)blockIdx.x * 256 + threadIdx.x; i < n16; i += (uint64_t)gridDim.x * 256) {
        const uint4 x = a[i];
        acc += x.x ^ x.y ^ x.z ^ x.w;
    }
    if (acc == 0x123456789ull) out[0] = 1;
}

int main()
{
    const uint64_t G = 1ull << 26;
    const int REPS = 10;
    int ncu = 0;
    CK(hipDeviceGetAttribute(&ncu, hipDeviceAttributeMultiprocessorCount, 0));
    uint8_t *buf[8];
    const uint64_t sz[8] = { 64 * G, 8 * R * G, 8 * R * G, R * G, R * G, G, G, 8 * G };
    for (int k = 0; k < 8; ++k) {
        CK(hipMalloc(&buf[k], sz[k]));
        CK(hipMemset(buf[k], k + 1, sz[k]));
    }
    hipLaunchKernelGGL(init_state, dim3(1024), dim3(256), 0, 0, (uint4 *)buf[0], G);
    CK(hipDeviceSynchronize());
    uint8_t *one;
    CK(hipMalloc(&one, kPerGroup * G));
    CK(hipMemset(one, 7, kPerGroup * G));
    uint32_t *out;
    CK(hipMalloc(&out, 4));
    Outs os;
    CK(hipMalloc(&os.med, 8 * G));
    CK(hipMalloc(&os.nh, 8 * G));
    CK(hipMalloc(&os.mn, 8 * G));
    CK(hipMalloc(&os.ah, G));
    CK(hipMalloc(&os.row, 32 * G));
    Cols c = { (const uint4 *)buf[0], (const uint64_t *)buf[1], (const uint64_t *)buf[2], buf[3], buf[4], buf[5], buf[6],
               (const uint64_t *)buf[7] };
    hipEvent_t e0, e1;
    CK(hipEventCreate(&e0));
    CK(hipEventCreate(&e1));
    const double bytes = (double)kPerGroup * G;
    for (int per_cu = 2; per_cu <= 8; per_cu *= 2) {
        const uint32_t grid = per_cu * ncu;
        for (int kind = 0; kind < 9; ++kind) {
            auto launch = [&]() {
                if (kind == 0) hipLaunchKernelGGL(cols_lane, dim3(grid), dim3(256), 0, 0, c, G, out);
                else if (kind == 1) hipLaunchKernelGGL(cols_wave, dim3(grid), dim3(256), 0, 0, c, G, out);
                else if (kind == 2) hipLaunchKernelGGL(one_stream, dim3(grid), dim3(256), 0, 0, (const uint4 *)one, kPerGroup * G / 16, out);
                else if (kind == 3) hipLaunchKernelGGL(lane_st<false>, dim3(grid), dim3(256), 0, 0, c, os, G);
                else if (kind == 4) hipLaunchKernelGGL(lane_st<true>, dim3(grid), dim3(256), 0, 0, c, os, G);
                else if (kind == 5) hipLaunchKernelGGL((lane_st<false, 3>), dim3(grid), dim3(256), 0, 0, c, os, G);
                else if (kind == 6) hipLaunchKernelGGL((lane_st<false, 2>), dim3(grid), dim3(256), 0, 0, c, os, G);
                else if (kind == 7) hipLaunchKernelGGL((lane_st<false, 1>), dim3(grid), dim3(256), 0, 0, c, os, G);
                else hipLaunchKernelGGL((lane_st<false, 0>), dim3(grid), dim3(256), 0, 0, c, os, G);
            };
            launch();
            CK(hipDeviceSynchronize());
            CK(hipEventRecord(e0, 0));
            for (int r = 0; r < REPS; ++r) launch();
            CK(hipEventRecord(e1, 0));
            CK(hipEventSynchronize(e1));
            float ms = 0;
            CK(hipEventElapsedTime(&ms, e0, e1));
            ms /= REPS;
            static const char *names[9] = { "cols_lane", "cols_wave", "one_stream", "lane_st", "lane_st_cmp",
                                            "lane_st_3out", "lane_st_2out", "lane_st_1out", "lane_st_row" };
            static const double wr[9] = { 0, 0, 0, 25, 25, 24, 16, 8, 32 };   // bytes written per group
            const double by = bytes + wr[kind] * G;
            printf("{\"kernel\": \"%s\", \"blocks_per_cu\": %d, \"ms\": %.4f, \"GBps\": %.1f}\n", names[kind], per_cu, ms,
                   by / ms / 1e6);
        }
    }
    return 0;
}
