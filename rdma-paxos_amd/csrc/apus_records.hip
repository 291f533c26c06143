// The proxy's stable-storage records -- the BDB record format
// -- for gfx950.  Semantics in include/apus_gpu.h (apus_records_*).
//
//   records_store_kernel  stablestorage_save_request (src/proxy/proxy.c:
//       269-291) on every entry persist_new_entries walks (src/dare/
//       dare_server.c:1792-1810): 16 lanes per group follow its chain from
//       the cursor (speculatively, below) and append each record to the
//       group's dump (store_record, src/db/db-interface.c:65-95, DB_APPEND).
//   records_load_kernel   stablestorage_load_records (proxy.c:306-336): 16
//       lanes per snapshot walk its records speculatively (below) and emit the
//       replay plan.
//
// Both are chains (an entry's or a record's length comes from its own header):
// a lane per chain walked 64 chains per wave one link per step (store 4.64
// ms, load 3.34 ms at C2 size); 16-lane segments confirm up to 16 links per
// step when the lengths repeat, as they do in a log of equal-size commands.
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

// ---- one lane per chain (APUS_BATCH_LANE_IMPL): the second implementation
// the segment kernels are cross-checked against.  The segments are faster
// even where lengths vary (C3: store 13.5 vs 15.1 ms, load 0.24 vs 0.90 ms) --
// a lane-per-chain walk there is bound by the TLB misses of 2^18 chains
// hopping through 88 GB ----
__global__ void __launch_bounds__(256) records_store_lane_kernel(const apus_batch_t b, const apus_records_io_t io,
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
        bool bad = !(len >= kHdr && len <= ring_cap(b) && end <= len && oe <= len);
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

__global__ void __launch_bounds__(256) records_load_lane_kernel(const apus_records_load_io_t io)
{
    for (uint64_t k = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x; k < io.n;
         k += (uint64_t)gridDim.x * blockDim.x) {
        const uint8_t *d = io.dump + k * io.stride;
        // a size beyond the dump's stride would read the next dump (or past
        // the array): the walk sees at most stride bytes
        const uint32_t size = (uint32_t)min((uint64_t)io.size[k], io.stride);
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

// ---- 16 lanes per chain (the default) ----
__device__ __forceinline__ uint32_t seg_bits(uint64_t ballot, uint32_t seg) { return (uint32_t)(ballot >> (16 * seg)) & 0xFFFFu; }

// one record's bytes from the entry at src to dst (24-B records of 8-B
// aligned entries as three u64)
__device__ __forceinline__ void rec_copy(uint8_t *dst, const uint8_t *src, uint32_t nb)
{
    if (nb == APUS_REC_SEND_BYTES && ((((uintptr_t)src) | ((uintptr_t)dst)) & 7u) == 0) {
        const uint64_t *s8 = reinterpret_cast<const uint64_t *>(src);
        uint64_t *d8 = reinterpret_cast<uint64_t *>(dst);
        const uint64_t w0 = s8[0], w1 = s8[1], w2 = s8[2];
        d8[0] = w0;
        d8[1] = w1;
        d8[2] = w2;
    } else if (((((uintptr_t)src) | ((uintptr_t)dst) | nb) & 3u) == 0) {
        for (uint32_t j = 0; j < nb; j += 4)
            *reinterpret_cast<uint32_t *>(dst + j) = *reinterpret_cast<const uint32_t *>(src + j);
    } else {
        for (uint32_t j = 0; j < nb; ++j) dst[j] = src[j];
    }
}

// persist_new_entries' walk + stablestorage_save_request, 16 lanes per group
// (four groups per wave): the entry chain is walked speculatively as in
// commit_seg_kernel -- lane j of a segment takes the entry at oe + j*el, el
// the last entry's length, and the segment's ballot bits confirm the longest
// prefix of entries of that length (plus the first of another length) that
// need no wrap, are not the end and whose records fit the log and the dump.
// The confirmed lanes place their records by a segment prefix sum and copy
// them side by side.  The wrap rules (header wrap, ghost header) and the
// stops are decided at the segment's first entry, exactly as the one-lane
// walk does.
__global__ void __launch_bounds__(256) records_store_kernel(const apus_batch_t b, const apus_records_io_t io,
                                                            uint64_t *stats)
{
    const uint32_t lane = lane_id();
    const uint32_t seg = lane >> 4, sl = lane & 15u;
    const uint64_t nseg = (uint64_t)gridDim.x * (blockDim.x >> 4);
    uint64_t corrupt = 0;
    for (uint64_t g0 = ((uint64_t)blockIdx.x * blockDim.x + (threadIdx.x & ~63u)) >> 4; g0 < b.n_groups;
         g0 += nseg) {
        const uint64_t g = g0 + seg;
        const bool live = g < b.n_groups;
        const uint64_t gc = live ? g : 0;
        const apus_group_state_t st = load_state(b, gc);
        const uint64_t end = st.end, len = st.len, cap = io.cap;
        const uint8_t *ring = b.ring + gc * b.ring_stride;
        uint8_t *dump = io.dump + gc * cap;
        uint64_t oe = io.cursor[gc], dl = io.dump_len[gc];
        uint32_t n = 0, elg = 128;
        const bool invalid = live && !(len >= kHdr && len <= ring_cap(b) && end <= len && oe <= len);
        bool bad = invalid;
        bool done = !live || bad;
        const uint64_t guard = len / kHdr + 4;
        uint64_t steps = 0;
        while (__ballot(!done)) {
            // the segment's first entry: log_offset_end_distance, log_get_entry's header wrap
            // (a walk of more than guard entries -- a corrupt log the reference
            // would never leave -- stops where the one-lane walk stops)
            if (!done) {
                if (dist(end, len, oe) == 0) done = true;
                else if (steps >= guard) { bad = true; done = true; }
                else if (len - oe < kHdr) oe = 0;
            }
            const uint64_t p = oe + (uint64_t)sl * elg;
            const bool hdr = !done && p <= len && len - p >= kHdr && (sl == 0 || p != end) && sl < guard - steps;
            uint32_t el = 0, nb = 0;
            const uint8_t *e = ring + (hdr ? p : 0);
            if (hdr) {
                const uint32_t type = e[kType];
                el = entry_len(type, ld_u16(e + kData));
                nb = type == 4u || type == 6u ? APUS_REC_CONNECT_BYTES
                     : type == 5u ? APUS_REC_SEND_BYTES + ld_u16(e + 24 + APUS_REC_DATA_OFF) : 0u;
            }
            const bool fit = hdr && len - p >= el;                       // log_fit_entry
            // the record's place: the segment's exclusive prefix of record bytes
            const uint32_t pre = row_scan_incl(fit ? nb : 0u);     // (a segment is a DPP row)
            const uint32_t ex = pre - (fit ? nb : 0u);
            const bool rec_ok = nb == 0 || (24u + (uint64_t)nb <= len - p && dl + ex + nb <= cap);
            const bool ok = fit && rec_ok;
            const bool cont = ok && el == elg && sl < 15u;
            const uint32_t okb = seg_bits(__ballot(ok), seg);
            const uint32_t fb = (uint32_t)__builtin_ctz(seg_bits(__ballot(!cont), seg) | 0x10000u);
            const uint32_t nconf = fb + ((okb >> fb) & 1u);
            const bool fit0 = __shfl(fit ? 1 : 0, lane & ~15u) != 0;
            if (!done && nconf == 0) {
                if (!fit0) {                                              // ghost header: the entry restarts at 0
                    oe = 0;
                    ++steps;
                } else {                                                  // the record: past the log or the dump
                    bad = true;
                    done = true;
                }
                continue;
            }
            const bool conf = !done && sl < nconf;
            if (conf && nb) rec_copy(dump + dl + ex, e + 24, nb);
            if (!done) {
                const uint32_t last = (lane & ~15u) + nconf - 1u;
                const uint64_t p_last = ((uint64_t)(uint32_t)__shfl((int)(uint32_t)(p >> 32), last) << 32) |
                                        (uint32_t)__shfl((int)(uint32_t)p, last);
                const uint32_t el_last = __shfl(el, last);
                oe = p_last + el_last;
                elg = el_last;
                dl += __shfl(pre, last);
                n += __builtin_popcount(seg_bits(__ballot(conf && nb != 0), seg));
                steps += nconf;
            }
        }
        if (live && sl == 0) {
            if (!invalid) {
                io.cursor[g] = oe;
                io.dump_len[g] = (uint32_t)dl;
            }
            if (io.n_records) io.n_records[g] = n;
        }
        if (live && sl == 0 && bad) ++corrupt;
    }
    if (corrupt) atomicAdd((unsigned long long *)&stats[APUS_STAT_CORRUPT], (unsigned long long)corrupt);
}

// stablestorage_load_records, 16 lanes per snapshot (four per wave): the
// walk is a chain -- a record's length comes from its own header -- so lane j
// of a segment reads the record at len + j*rl, rl the last record's length
// (24 B for a SEND of an R <= 4 log), and the segment's 16 ballot bits confirm
// the longest prefix of records of that length, plus the first record of
// another length: one step covers up to 16 records, their plan entries
// written as one coalesced 256-B row.  A record that cannot be replayed
// (unknown action, past the snapshot) ends the chain before it; when it is
// the segment's first, the walk stops there with the reference's status.
__global__ void __launch_bounds__(256) records_load_kernel(const apus_records_load_io_t io)
{
    const uint32_t lane = lane_id();
    const uint32_t seg = lane >> 4, sl = lane & 15u;
    const uint64_t nseg = (uint64_t)gridDim.x * (blockDim.x >> 4);
    for (uint64_t k0 = ((uint64_t)blockIdx.x * blockDim.x + (threadIdx.x & ~63u)) >> 4; k0 < io.n; k0 += nseg) {
        const uint64_t k = k0 + seg;                       // this segment's snapshot
        const bool live = k < io.n;
        const uint8_t *d = io.dump + (live ? k : 0) * io.stride;
        const uint32_t size = live ? (uint32_t)min((uint64_t)io.size[k], io.stride) : 0u;   // (as above)
        uint32_t len = 0, n = 0, rl = APUS_REC_SEND_BYTES, status = 0;
        uint32_t c0 = 0, c1 = 0, c2 = 0;
        bool done = !live || size == 0;
        while (__ballot(!done)) {
            // lane j: can the record at p be replayed, and its length
            // (in 64 bits: len + 15 * rl may pass 2^32 when size is near 4 GiB)
            const uint64_t p64 = (uint64_t)len + (uint64_t)sl * rl;
            const uint32_t room = p64 < size ? size - (uint32_t)p64 : 0u;
            const uint32_t p = (uint32_t)p64;                 // used only when room > 0 (p < size)
            uint32_t action = 0, conn = 0, rb = 0, dlen = 0, why = 2;   // why: 0 ok, 1 unknown, 2 past size
            if (!done && room >= APUS_REC_CONNECT_BYTES) {
                const uint8_t *r = d + p;
                if ((((uintptr_t)r) & 3u) == 0) {
                    const uint32_t w = *reinterpret_cast<const uint32_t *>(r);
                    conn = w & 0xFFFFu;
                    action = (w >> 16) & 0xFFu;
                } else {
                    conn = ld_u16(r);
                    action = r[2];
                }
                if (action == 5u) {
                    if (room >= APUS_REC_DATA_OFF + 2) {
                        dlen = ld_u16(r + APUS_REC_DATA_OFF);
                        rb = APUS_REC_SEND_BYTES + dlen;
                        why = rb <= room ? 0u : 2u;
                    }
                } else if (action == 4u || action == 6u) {
                    rb = APUS_REC_CONNECT_BYTES;
                    why = 0;
                } else {
                    why = 1;
                }
            }
            const bool ok = !done && why == 0;
            const bool cont = ok && rb == rl && sl < 15u;
            const uint32_t okb = seg_bits(__ballot(ok), seg);
            const uint32_t fb = (uint32_t)__builtin_ctz(seg_bits(__ballot(!cont), seg) | 0x10000u);
            const uint32_t nconf = fb + ((okb >> fb) & 1u);
            // the segment's first record decides a stop
            const uint32_t why0 = __shfl(why, lane & ~15u);
            if (!done && nconf == 0) {
                status = why0;
                done = true;
            }
            const bool conf = !done && sl < nconf;
            if (conf && io.plan && n + sl < io.max_plan) {
                uint4 e;
                e.x = p;
                e.y = dlen;
                e.z = conn | (action << 16);
                e.w = 0;
                *reinterpret_cast<uint4 *>(io.plan + k * io.max_plan + n + sl) = e;
            }
            c0 += conf && action == 4u;
            c1 += conf && action == 5u;
            c2 += conf && action == 6u;
            if (!done) {
                const uint32_t last = (lane & ~15u) + nconf - 1u;
                const uint32_t p_last = __shfl(p, last), rb_last = __shfl(rb, last);
                len = p_last + rb_last;
                rl = rb_last;
                n += nconf;
                if (len >= size) done = true;
            }
        }
        // per-segment sums of the action counts (a segment is a DPP row)
#pragma unroll
        for (int dd = 1; dd < 16; dd <<= 1) {
            c0 += __shfl_xor(c0, dd);
            c1 += __shfl_xor(c1, dd);
            c2 += __shfl_xor(c2, dd);
        }
        if (live && sl == 0) {
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
}

hipError_t launch_records_store(apus_ctx *ctx, const apus_batch_t &b, const apus_records_io_t &io, hipStream_t s)
{
    if (!b.n_groups) return hipSuccess;
    if (b.flags & APUS_BATCH_LANE_IMPL) {
        const uint32_t grid = grid_for(b.n_groups, 256, ctx->n_cu, 8);
        hipLaunchKernelGGL(records_store_lane_kernel, dim3(grid), dim3(256), 0, s, b, io, ctx->stats);
        return hipGetLastError();
    }
    const uint32_t grid = grid_for(b.n_groups, 16, ctx->n_cu, 8);      // 16 groups per 256-thread block
    hipLaunchKernelGGL(records_store_kernel, dim3(grid), dim3(256), 0, s, b, io, ctx->stats);
    return hipGetLastError();
}

hipError_t launch_records_load(apus_ctx *ctx, const apus_records_load_io_t &io, hipStream_t s)
{
    if (!io.n) return hipSuccess;
    if (io.flags & APUS_BATCH_LANE_IMPL) {
        const uint32_t grid = grid_for(io.n, 256, ctx->n_cu, 8);
        hipLaunchKernelGGL(records_load_lane_kernel, dim3(grid), dim3(256), 0, s, io);
        return hipGetLastError();
    }
    const uint32_t grid = grid_for(io.n, 16, ctx->n_cu, 8);          // 16 snapshots per 256-thread block
    hipLaunchKernelGGL(records_load_kernel, dim3(grid), dim3(256), 0, s, io);
    return hipGetLastError();
}

}  // namespace apus
