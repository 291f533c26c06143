// The proxy's stable-storage records -- the BDB record format
// -- for gfx950.  Semantics in include/apus_gpu.h (apus_records_*).
//
//   records_store_kernel  stablestorage_save_request (src/proxy/proxy.c:
//       269-291) on every entry persist_new_entries walks (src/dare/
//       dare_server.c:1792-1810): one LANE per group follows its chain from
//       the cursor and appends each record to the group's dump (store_record,
//       src/db/db-interface.c:65-95, DB_APPEND).
//   records_load_kernel   stablestorage_load_records (proxy.c:306-336): one
//       LANE per snapshot walks its records and emits the replay plan.
//
// Both are chains of dependent reads of a few bytes (a record's length comes
// from its own header), so a lane per chain keeps 64 independent chains in
// flight per wave.  Records of 4 and 24 B keep a dump 4-B aligned: they move
// as dwords when source and destination allow it.
#include "apus_device.h"
#include "apus_internal.h"

namespace apus {

__device__ __forceinline__ uint32_t rec_bytes(const uint8_t *e)
{
    const uint32_t action = e[kType];                        // proxy_msg_header.action = entry type@26
    if (action == 4u || action == 6u) return APUS_REC_CONNECT_BYTES;
    if (action == 5u) return APUS_REC_SEND_BYTES + ld_u16(e + 24 + APUS_REC_DATA_OFF);   // data.cmd.len @ entry+32
    return 0u;
}

__global__ void __launch_bounds__(256) records_store_kernel(const apus_batch_t b, const apus_records_io_t io,
                                                            uint64_t *stats)
{
    uint64_t corrupt = 0;
    for (uint64_t g = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x; g < b.n_groups;
         g += (uint64_t)gridDim.x * blockDim.x) {
        const apus_group_state_t st = load_state(b, g);
        const uint64_t end = st.end, len = st.len, cap = io.cap;
        const uint8_t *ring = b.ring + g * b.ring_stride;
        uint8_t *dump = io.dump + g * cap;
        uint64_t oe = io.cursor[g], dl = io.dump_len[g];
        uint32_t n = 0;
        bool bad = !(len >= kHdr && len <= b.ring_stride && end <= len && oe <= len);
        if (!bad) {
            const uint64_t guard = len / kHdr + 4;
            uint64_t steps = 0;
            // while (log_is_offset_larger(log, log->end, log->old_end))
            while (dist(end, len, oe) != 0) {
                if (++steps > guard) { bad = true; break; }
                if (len - oe < kHdr) oe = 0;                      // log_get_entry
                const uint8_t *e = ring + oe;
                const uint8_t *src = e + 24;
                uint8_t *dst = dump + dl;
                // an 8-B aligned entry: bytes 24..47 (the record of a CONNECT /
                // CLOSE / 24-B SEND, type@26 and data.cmd.len@32 among them)
                // as three u64 loads, and cmd.len@48 as one u16
                const bool al8 = ((((uintptr_t)src) | ((uintptr_t)dst)) & 7u) == 0;
                uint64_t w0 = 0, w1 = 0, w2 = 0;
                uint32_t type, nb;
                if (al8) {
                    const uint64_t *s8 = reinterpret_cast<const uint64_t *>(src);
                    w0 = s8[0];
                    w1 = s8[1];
                    w2 = s8[2];
                    type = (uint32_t)(w0 >> 16) & 0xFFu;
                    nb = type == 4u || type == 6u ? APUS_REC_CONNECT_BYTES
                         : type == 5u ? APUS_REC_SEND_BYTES + ((uint32_t)w1 & 0xFFFFu) : 0u;
                } else {
                    type = e[kType];
                    nb = rec_bytes(e);
                }
                const uint32_t el = entry_len(type, ld_u16(e + kData));
                if (len - oe < el) { oe = 0; continue; }          // !log_fit_entry: ghost header
                if (nb) {
                    if (24u + (uint64_t)nb > len - oe || dl + nb > cap) { bad = true; break; }
                    if (al8 && nb == APUS_REC_SEND_BYTES) {
                        uint64_t *d8 = reinterpret_cast<uint64_t *>(dst);
                        d8[0] = w0;
                        d8[1] = w1;
                        d8[2] = w2;
                    } else if (al8 && nb == APUS_REC_CONNECT_BYTES) {
                        *reinterpret_cast<uint32_t *>(dst) = (uint32_t)w0;
                    } else if (((((uintptr_t)src) | ((uintptr_t)dst) | nb) & 3u) == 0) {
                        for (uint32_t j = 0; j < nb; j += 4)
                            *reinterpret_cast<uint32_t *>(dst + j) = *reinterpret_cast<const uint32_t *>(src + j);
                    } else {
                        for (uint32_t j = 0; j < nb; ++j) dst[j] = src[j];
                    }
                    dl += nb;
                    ++n;
                }
                oe += el;
            }
            io.cursor[g] = oe;
            io.dump_len[g] = (uint32_t)dl;
        }
        if (io.n_records) io.n_records[g] = n;
        if (bad) ++corrupt;
    }
    if (corrupt) atomicAdd((unsigned long long *)&stats[APUS_STAT_CORRUPT], (unsigned long long)corrupt);
}

__global__ void __launch_bounds__(256) records_load_kernel(const apus_records_load_io_t io)
{
    for (uint64_t k = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x; k < io.n;
         k += (uint64_t)gridDim.x * blockDim.x) {
        const uint8_t *d = io.dump + k * io.stride;
        const uint32_t size = io.size[k];
        uint32_t len = 0, n = 0, c0 = 0, c1 = 0, c2 = 0, status = 0;
        while (len < size) {
            if (size - len < APUS_REC_CONNECT_BYTES) { status = 2; break; }   // header past size
            const uint8_t *r = d + len;
            uint32_t conn, action;
            if ((((uintptr_t)r) & 3u) == 0) {
                const uint32_t w = *reinterpret_cast<const uint32_t *>(r);
                conn = w & 0xFFFFu;
                action = (w >> 16) & 0xFFu;
            } else {
                conn = ld_u16(r);
                action = r[2];
            }
            uint32_t rb, dlen = 0;
            if (action == 5u) {                                               // SEND: PROXY_SEND_MSG_SIZE
                if (size - len < APUS_REC_DATA_OFF + 2) { status = 2; break; }
                dlen = ld_u16(r + APUS_REC_DATA_OFF);
                rb = APUS_REC_SEND_BYTES + dlen;
            } else if (action == 4u || action == 6u) {                       // CONNECT, CLOSE
                rb = APUS_REC_CONNECT_BYTES;
            } else {
                status = 1;                                                   // the reference never advances
                break;
            }
            if (rb > size - len) { status = 2; break; }                       // would read past the snapshot
            if (io.plan && n < io.max_plan) {
                uint32_t *p = reinterpret_cast<uint32_t *>(io.plan + k * io.max_plan + n);
                p[0] = len;
                p[1] = dlen;
                p[2] = conn | (action << 16);
                p[3] = 0;
            }
            ++n;
            c0 += action == 4u;
            c1 += action == 5u;
            c2 += action == 6u;
            len += rb;
        }
        io.n_records[k] = n;
        io.status[k] = status;
        if (io.stop) io.stop[k] = len;
        if (io.counts) {
            io.counts[3 * k] = c0;
            io.counts[3 * k + 1] = c1;
            io.counts[3 * k + 2] = c2;
        }
    }
}

hipError_t launch_records_store(apus_ctx *ctx, const apus_batch_t &b, const apus_records_io_t &io, hipStream_t s)
{
    if (!b.n_groups) return hipSuccess;
    const uint32_t grid = grid_for(b.n_groups, 256, ctx->n_cu, 8);
    hipLaunchKernelGGL(records_store_kernel, dim3(grid), dim3(256), 0, s, b, io, ctx->stats);
    return hipGetLastError();
}

hipError_t launch_records_load(apus_ctx *ctx, const apus_records_load_io_t &io, hipStream_t s)
{
    if (!io.n) return hipSuccess;
    const uint32_t grid = grid_for(io.n, 256, ctx->n_cu, 8);
    hipLaunchKernelGGL(records_load_kernel, dim3(grid), dim3(256), 0, s, io);
    return hipGetLastError();
}

}  // namespace apus
