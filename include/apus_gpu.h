/*
 * libapus_gpu — MI355X (gfx950) engine for the quorum / commit hot path of
 * APUS (DARE + proxy), wnagchenghku/RDMA-PAXOS.
 *
 * C ABI only: plain C structs, plain pointers and sizes, no C++ or torch types.
 * Every entry point cites the reference code whose semantics it reproduces
 * bit-exactly (paths relative to the reference tree's root).
 *
 * Two families of entry points:
 *   1. Scalar drop-ins that take the reference's own structs by pointer
 *      (dare_log_t, server_config_t, ctrl_data_t), for the single DARE event
 *      loop thread.  They run the same HIP kernels as the batched API with
 *      one group (G = 1) on the library's default context.
 *   2. Batched, stream-ordered entry points over millions of independent
 *      consensus groups whose state is resident in HBM (group-major arrays).
 *
 * Return codes mirror the reference (src/dare/dare_ibv_rc.c:27-29,
 * src/include/dare/debug.h:75): APUS_OK (0) success, APUS_ERROR (1) hard
 * error, APUS_INSUCCESS (-1) "not yet / retry".  No errno, no exceptions;
 * errors are optionally printed to a caller supplied FILE* (apus_set_log).
 *
 * Ownership: the caller owns every buffer.  The library never frees or
 * reallocates caller memory; scalar calls copy the bytes they need into
 * library-owned device scratch (no allocation per call after the first).
 */
#ifndef APUS_GPU_H
#define APUS_GPU_H

#include <stdint.h>
#include <stddef.h>
#include <stdio.h>

#ifdef __cplusplus
extern "C" {
#endif

/* ------------------------------------------------------------------------ */
/* Constants (values identical to the reference)                             */
/* ------------------------------------------------------------------------ */
#define APUS_OK          0
#define APUS_ERROR       1
#define APUS_INSUCCESS (-1)

#define APUS_MAX_SERVER_COUNT 13          /* src/include/dare/dare.h:26        */
#define APUS_MAX_NC_ENTRIES   1024        /* src/include/dare/dare_log.h:60    */
#define APUS_ENTRY_HDR        64          /* sizeof(dare_log_entry_t)          */

/* entry types: src/include/dare/dare_log.h:21-24; APUS proxy actions
 * CONNECT/SEND/CLOSE = 4/5/6 (src/include/proxy/proxy.h:10-12) are CSM-class */
#define APUS_NOOP    0
#define APUS_CSM     1
#define APUS_CONFIG  2
#define APUS_HEAD    3

/* configuration states: src/include/dare/dare_config.h:17-28 */
#define APUS_CID_STABLE    0
#define APUS_CID_TRANSIT   1
#define APUS_CID_EXTENDED  2

/* log replication steps: src/include/dare/dare_server.h:78-84 */
#define APUS_LR_GET_WRITE    1
#define APUS_LR_GET_NCE_LEN  2
#define APUS_LR_GET_NCE      3
#define APUS_LR_SET_END      4
#define APUS_LR_UPDATE_LOG   5
#define APUS_LR_UPDATE_END   6
#define APUS_PERMANENT_FAILURE 2          /* src/include/dare/dare_server.h:76 */

/* ------------------------------------------------------------------------ */
/* Byte-compatible mirrors of the reference structs (x86-64 SysV layout).    */
/* tests/test_abi.py checks every offset against the reference headers.      */
/* ------------------------------------------------------------------------ */

/* dare_cid_t, src/include/dare/dare_config.h:38-45 (16 B) */
typedef struct apus_cid {
    uint64_t epoch;
    uint8_t  size[2];
    uint8_t  state;
    uint8_t  pad[1];
    uint32_t bitmask;
} apus_cid_t;

/* dare_log_entry_t, src/include/dare/dare_log.h:33-48 (64 B header; a CSM
 * entry's command bytes start at data.cmd.cmd (offset 50) and run past the
 * header: log_entry_len = 64 + cmd.len, dare_log.h:228-234). */
typedef struct apus_log_entry {
    uint64_t idx;                         /* @0  */
    uint64_t term;                        /* @8  */
    uint64_t req_id;                      /* @16 */
    uint16_t clt_id;                      /* @24 */
    uint8_t  type;                        /* @26 */
    uint8_t  sender;                      /* @27 */
    uint8_t  reply[APUS_MAX_SERVER_COUNT];/* @28 */
    union {
        struct { uint16_t len; uint8_t cmd[14]; } cmd;  /* @48 (sm_cmd_t)  */
        apus_cid_t cid;
        uint64_t   head;
    } data;                               /* @48 */
} apus_log_entry_t;

/* dare_log_entry_det_t, dare_log.h:51-56 (24 B) */
typedef struct apus_entry_det {
    uint64_t idx;
    uint64_t term;
    uint64_t offset;
} apus_entry_det_t;

/* dare_nc_buf_t, dare_log.h:60-65 (24,584 B) */
typedef struct apus_nc_buf {
    uint64_t len;
    apus_entry_det_t entries[APUS_MAX_NC_ENTRIES];
} apus_nc_buf_t;

/* dare_log_t, dare_log.h:77-103 (header 319,656 B, then the ring) */
typedef struct apus_log {
    uint64_t head, apply, commit, end, tail, old_end, old_commit, len;
    apus_nc_buf_t nc_buf[APUS_MAX_SERVER_COUNT];
    uint8_t entries[];
} apus_log_t;

/* server_t, src/include/dare/dare_server.h:86-95 (40 B) */
typedef struct apus_server {
    uint64_t next_wr_id;
    uint64_t cached_end_offset;
    uint64_t last_get_read_ssn;
    void    *ep;
    uint8_t  fail_count;
    uint8_t  next_lr_step;
    uint8_t  send_flag;
    uint8_t  send_count;
} apus_server_t;

/* server_config_t, src/include/dare/dare_config.h:59-75 (56 B) */
typedef struct apus_server_config {
    apus_cid_t     cid;
    uint64_t       cid_offset;
    uint64_t       cid_idx;
    uint64_t       req_id;
    apus_server_t *servers;
    uint16_t       clt_id;
    uint8_t        idx;
    uint8_t        len;
} apus_server_config_t;

/* vote_req_t, dare_server.h:99-105 (40 B) */
typedef struct apus_vote_req {
    uint64_t   sid;
    uint64_t   index;
    uint64_t   term;
    apus_cid_t cid;
} apus_vote_req_t;

/* log_offsets_t, dare_log.h:67-73 */
typedef struct apus_log_offsets {
    uint64_t head, apply, commit, end;
} apus_log_offsets_t;

/* sm_rep_t, dare_server.h:115-120 */
typedef struct apus_sm_rep {
    uint64_t sid, raddr;
    uint32_t rkey, len;
} apus_sm_rep_t;

/* ctrl_data_t, dare_server.h:123-140 (1,880 B) */
typedef struct apus_ctrl_data {
    uint64_t           sid;
    apus_vote_req_t    vote_req[APUS_MAX_SERVER_COUNT];
    apus_log_offsets_t log_offsets[APUS_MAX_SERVER_COUNT];
    apus_sm_rep_t      sm_rep[APUS_MAX_SERVER_COUNT];
    uint64_t           sm_req[APUS_MAX_SERVER_COUNT];
    uint64_t           hb[APUS_MAX_SERVER_COUNT];
    uint64_t           vote_ack[APUS_MAX_SERVER_COUNT];
    uint64_t           rsid[APUS_MAX_SERVER_COUNT];
    uint64_t           apply_offsets[APUS_MAX_SERVER_COUNT];
    uint64_t           prv_data[APUS_MAX_SERVER_COUNT];
} apus_ctrl_data_t;

/* ------------------------------------------------------------------------ */
/* Batched layout (device-resident, group-major)                             */
/* ------------------------------------------------------------------------ */

/* One group's log offsets + configuration: the dare_log_t header fields the
 * hot path reads (dare_log.h:79-95) plus config.cid.  64 B, AoS. */
typedef struct apus_group_state {
    uint64_t   head, apply, commit, end, tail, len;
    apus_cid_t cid;
} apus_group_state_t;

/* Descriptor of a batch of G groups.  All pointers are DEVICE pointers.
 * ring:    G rings of ring_stride bytes (ring_stride % 16 == 0, >= len);
 *          group g's dare_log_t.entries[] image is ring[g*ring_stride ...].
 * Per-replica arrays are [G][n_replicas] (row-major, server index i is the
 * column, exactly the reference's [MAX_SERVER_COUNT] arrays truncated to
 * n_replicas).  A NULL per-replica pointer is allowed when the entry point
 * called does not read that array. */
typedef struct apus_batch {
    uint64_t n_groups;
    uint32_t n_replicas;        /* <= APUS_MAX_SERVER_COUNT                  */
    uint32_t flags;             /* APUS_BATCH_* (0 = defaults)               */
    uint64_t ring_stride;
    uint8_t            *ring;
    apus_group_state_t *state;         /* [G]                                */
    uint8_t            *self_idx;      /* [G]     config.idx                 */
    uint64_t           *remote_end;    /* [G][R]  ctrl->log_offsets[i].end   */
    uint64_t           *remote_commit; /* [G][R]  ctrl->log_offsets[i].commit*/
    uint8_t            *lr_step;       /* [G][R]  servers[i].next_lr_step    */
    uint8_t            *fail_count;    /* [G][R]  servers[i].fail_count      */
    uint64_t           *vote_ack;      /* [G][R]  ctrl->vote_ack[i]          */
    uint64_t           *apply_offsets; /* [G][R]  ctrl->apply_offsets[i]     */
    apus_vote_req_t    *vote_req;      /* [G][R]  ctrl->vote_req[i]          */
    uint64_t           *hb;            /* [G][R]  ctrl->hb[i]                */
    uint64_t           *sid;           /* [G]     ctrl->sid                  */
    uint64_t           *last_idx_term; /* [G][2]  local last entry (idx,term)*/
    uint8_t            *prev_head;     /* [G]     prev_log_entry_head        */
    uint64_t           *abs_base;      /* [G]     absolute position of ring
                                          offset 0 (wraps*len), for the
                                          cross-group pruning watermark      */
    apus_cid_t         *cid;           /* [G]     config.cid (APUS_BATCH_LOG_IMAGE
                                          only; else state[g].cid is used)    */
    uint16_t           *rc_connected;  /* [G]     bit i = servers[i].ep->
                                          rc_connected (NULL = all connected;
                                          read by APUS_COMMIT_PUBLISH)        */
    uint64_t           *vote_sit;      /* [G][R][3] optional (ABI 6): vote_req[i]'s
                                          sid, index, term -- the 24 B of each
                                          40-B record the ranking compares --
                                          packed; when set, the ranking reads
                                          these instead of the records (168 B per
                                          7-replica group instead of 280); vote_req
                                          is still read for the winner's cid.
                                          NULL: the records                  */
} apus_batch_t;

/* apus_batch_t.flags: run the commit walk with the one-lane-per-group kernel
 * (a second, independent implementation used to cross-check the default
 * wave-per-group LDS-window kernel). */
#define APUS_BATCH_LANE_IMPL 0x1u
/* apus_batch_t.flags: a performance hint for batches whose walks are short
 * (a span [commit, end) of at most 2,304 B at its 16-B phase, e.g. 16 entries
 * of 128 B): the commit walk runs four groups per wave, one per 16-lane
 * segment (commit_seg_kernel).  A group whose span does not fit is deferred to
 * the exact one-lane walk (APUS_STAT_SLOW counts it).  Results are identical
 * either way. */
#define APUS_BATCH_SHORT_WALKS 0x2u
/* apus_batch_t.flags: every group is a device-resident dare_log_t image
 * (dare_log.h:77-103) -- the reference's own RDMA-registered log layout,
 * header (head@0 apply@8 commit@16 end@24 tail@32 old_end@40 old_commit@48
 * len@56, nc_buf[13]@64) then entries[] at +APUS_LOG_HDR_BYTES -- so that
 * remote writes (a follower's reply[i] byte, rc_send_entries_reply,
 * dare_ibv_rc.c:1828-1863; the leader's end / entries writes) can land in
 * HBM and be read in place.  `ring` points at group 0's entries[] and
 * ring_stride is the image stride (header of group g at ring + g*stride -
 * APUS_LOG_HDR_BYTES); `state` is not read (may be NULL); `cid` [G] holds
 * config.cid.  Every entry point but apus_gen_batch accepts it; the writers
 * update the image in place as the reference updates its log: entries[] and
 * end/tail (apus_append_batch, log_append_entry), apply (apus_apply_batch),
 * head (apus_config_scan_batch), commit (apus_log_adjust_batch), and
 * config.cid in b->cid.  apus_persist_batch keeps its cursors in
 * apus_persist_in_t.old_end (one per replica copy).  The wave commit kernel
 * needs entries[] 16-B aligned (images at 8 mod 16). */
#define APUS_BATCH_LOG_IMAGE 0x4u
/* apus_batch_t.flags: a performance hint for batches whose entries vary in
 * length (e.g. memcached values of 64 B - 4 KB): the wave commit kernel may
 * then follow the entry chain one header per hop (three LDS byte reads)
 * instead of speculating that the next 64 entries have the last one's length,
 * and tallies the gathered entries in one lane-parallel pass.  Without it a
 * walk over entries of changing length confirms about one entry per wave
 * step.  Results are identical either way; fixed-size batches (C2) run the
 * kernel built without the hop path. */
#define APUS_BATCH_VAR_LEN 0x8u
/* apus_batch_t.flags: run apus_commit_batch's tail (median, pruning, publish,
 * forced pruning, failover pass) with eight lanes per group (quorum_row_kernel,
 * lane r = replica r) instead of the default one lane per group, for the
 * bench flag sets on checksum walks at R = 3, 5, 7.  Results are identical
 * either way; the row form measured slower (C5 tail 2.54 against 1.40 ms,
 * C2 0.11 against 0.05 ms: DESIGN 3.1g), and is kept as that A/B. */
#define APUS_BATCH_TAIL_ROWS 0x10u
#define APUS_LOG_HDR_BYTES 319656u        /* sizeof(dare_log_t) header      */

/* Outputs of apus_vote_batch (device). */
typedef struct apus_vote_out {
    uint8_t  *won;          /* [G] 1 = candidate won (dare_server.c:1362-1370) */
    uint8_t  *vote_count;   /* [G][2]                                          */
    uint64_t *new_commit;   /* [G] commit after max over vote_ack              */
    uint16_t *voters;       /* [G] bitmask of i whose vote_ack counted
                               (they get log_offsets[i].commit = vote_ack[i]
                                and next_lr_step = LR_GET_NCE_LEN)            */
} apus_vote_out_t;

/* Outcome codes of the voter-side ranking (dare_server.c:1526-1655). */
#define APUS_RANK_LEADER_KNOWN  0  /* own SID has L set: ignore requests     */
#define APUS_RANK_ADOPT_HB      1  /* hb[possible_leader] has same term      */
#define APUS_RANK_NO_BETTER     2  /* no request SID beats [TERM|1|IDX]      */
#define APUS_RANK_RAISE_TERM    3  /* local log best; new_sid = raised term  */
#define APUS_RANK_VOTE          4  /* vote: new_sid = candidate SID          */

typedef struct apus_rank_out {
    uint8_t    *outcome;    /* [G] APUS_RANK_*                                 */
    uint64_t   *new_sid;    /* [G] SID the voter proposes to install           */
    apus_cid_t *new_cid;    /* [G] candidate cid (APUS_RANK_VOTE only)         */
    uint16_t   *cleared;    /* [G] bitmask of vote_req[i].sid set to 0         */
} apus_rank_out_t;

/* Outcome of force_log_pruning for a group (dare_server.c:2069-2122). */
#define APUS_FORCE_NONE    0   /* log_size < 0.75 * len: nothing pruned          */
#define APUS_FORCE_PRUNE   1   /* log_pruning: the slowest server is the leader
                                  (target == self) or OFF in cid                 */
#define APUS_FORCE_REMOVE  2   /* the slowest server was removed (CID_SERVER_RM,
                                  req_id = clt_id = 0, a CONFIG entry appended,
                                  dare_ib_disconnect_server(target)), then
                                  log_pruning                                    */
#define APUS_FORCE_REFUSED 3   /* REMOVE's CONFIG append meets offsets the batched
                                  append refuses (a corrupt log; undefined in the
                                  reference): nothing is changed -- no removal, no
                                  append, no log_pruning (outputs as for NONE,
                                  target set); APUS_STAT_CORRUPT counts it       */

typedef struct apus_force_out {
    uint8_t  *action;      /* [G] APUS_FORCE_*                                   */
    uint8_t  *target;      /* [G] the server with the smallest apply offset
                              (config.idx when none is smaller than the leader's) */
    uint64_t *cfg_idx;     /* [G] REMOVE: log_append_entry's return for the
                              CONFIG entry (0: the log was full); else 0         */
    uint64_t *req_id;      /* [G] in/out data.config.req_id (0 on REMOVE), or NULL */
    uint16_t *clt_id;      /* [G] in/out data.config.clt_id (0 on REMOVE), or NULL */
} apus_force_out_t;

/* Outputs of apus_commit_batch (device pointers; NULL = not wanted). */
typedef struct apus_commit_out {
    uint64_t *new_commit;   /* [G] commit offset after the reply walk        */
    uint8_t  *committed;    /* [G] 1 if the commit advanced (the `committed`
                               flag, dare_ibv_rc.c:1744-1757), 0 if not,
                               0xFF if the walk hit the step guard (corrupt) */
    uint32_t *n_entries;    /* [G] entries walked and committed              */
    uint32_t *digest;       /* [G] Adler-32 of the walked entries' immutable
                               bytes (APUS_COMMIT_CHECKSUM; build-defined)   */
    uint64_t *median;       /* [G] DARE median-offset quorum result
                               (APUS_COMMIT_MEDIAN; dare_ibv_rc.c:1650-1723) */
    /* APUS_COMMIT_PRUNE: log_pruning's minimum in the same pass (a7,
     * dare_server.c:2026-2058) -- exactly apus_prune_batch's outputs, with the
     * OFF servers' apply offsets reset in place and the pruning watermark
     * (needs abs_base) folded into APUS_STAT_MIN_WATERMARK.                 */
    uint64_t *new_head;     /* [G] (NULL = not wanted)                       */
    uint8_t  *append_head;  /* [G]                                           */
    uint64_t *min_apply;    /* [G]                                           */
    /* APUS_COMMIT_NC: log_entries_to_nc_buf (a9, dare_log.h:339-359) of
     * [commit, end) from the same pass over the ring -- exactly what
     * apus_nc_build_batch writes: nc_dets [G][nc_max], nc_len [G].         */
    apus_entry_det_t *nc_dets;
    uint32_t *nc_len;
    uint32_t  nc_max;       /* determinants per group row (<= 2^31)          */
    uint32_t  pad;
    /* APUS_COMMIT_LAST_IT: [G][2] the local (idx, term) a candidate puts in its
     * vote request (poll_vote_requests, dare_server.c:1598-1620) -- exactly
     * what apus_last_idx_term_batch writes.                                  */
    uint64_t *last_idx_term;
    /* APUS_COMMIT_VOTE: poll_vote_count's tally (a5, dare_server.c:1330-1373)
     * of every group in the same tail pass -- exactly what apus_vote_batch
     * writes; votes won go to APUS_STAT_VOTES_WON.                           */
    apus_vote_out_t vote;
    /* APUS_COMMIT_RANK: poll_vote_requests' ranking (a6,
     * dare_server.c:1526-1655) in the same tail pass -- exactly what
     * apus_vote_rank_batch writes, on the local (idx, term) of
     * APUS_COMMIT_LAST_IT when that flag is set, else on b->last_idx_term.   */
    apus_rank_out_t rank;
    /* APUS_COMMIT_PUBLISH: the lazy remote-commit update that ends
     * update_remote_logs (dare_ibv_rc.c:1760-1822), on the commit the walk
     * leaves (or state.commit when the call does not walk): remote_commit is
     * updated in place and bit i of publish[g] is set for every server whose
     * 8-B commit write the leader posts (RDMA WRITE of remote_commit[g][i] to
     * the remote log->commit; the caller posts it).                          */
    uint16_t *publish;      /* [G]                                           */
    uint64_t *ssn;          /* [G] in/out the leader's ssn: +1 where publish[g]
                               != 0 (`if (!init) ssn++`, :1788-1789); NULL =
                               not kept                                       */
    /* APUS_COMMIT_FORCE_PRUNE: force_log_pruning (dare_server.c:2069-2122) in
     * the tail pass, after the publish, on the log as given (state.commit;
     * the flag is refused beside APUS_COMMIT_WALK / CHECKSUM: polling() runs
     * apply_committed_entries between the commit rule and force_log_pruning,
     * dare_server.c:1100-1123, and force_log_pruning starts from log->apply --
     * so the leader's poll is the commit call, log->commit = new_commit,
     * apus_apply_batch, then this).  It replaces APUS_COMMIT_PRUNE's
     * log_pruning: new_head / append_head / min_apply (when given) are
     * log_pruning's results where force_log_pruning calls it, and (head, 0,
     * 0) where it returns early (APUS_FORCE_NONE, APUS_FORCE_REFUSED).  On
     * REMOVE the group's cid (bitmask), ring, end, tail and prev_head are
     * updated in place by the CONFIG append (log_append_entry,
     * dare_log.h:466-558; term = SID_GET_TERM(sid), needs b->sid) and
     * apply_offsets[g][size] is set to apply (the reference writes
     * apply_offsets[i] with i == size after its loop, :2113; deviation:
     * skipped when size >= n_replicas, the batch has no such column).
     * Servers i >= n_replicas are never visited.                             */
    apus_force_out_t force;
} apus_commit_out_t;

/* One call runs the walk kernel, then ONE tail launch that walks the groups
 * the walk kernel deferred, computes the median and the pruning minimum of
 * every group from one read of its state row, and folds the statistics.   */
#define APUS_COMMIT_WALK      0x1u  /* a3: APUS reply-count commit walk    */
#define APUS_COMMIT_CHECKSUM  0x2u  /* a12: Adler-32 over [commit, end)     */
#define APUS_COMMIT_MEDIAN    0x4u  /* a4: DARE median quorum (lane/group)  */
/* a7: the pruning minimum (apus_prune_batch's work) in the same call.       */
#define APUS_COMMIT_PRUNE     0x8u
/* a9: the NC determinants of the walked range.  With APUS_COMMIT_CHECKSUM on
 * the wave kernel (or the lane kernel) they are written by the walk itself,
 * from the headers it already holds; otherwise by an apus_nc_build_batch
 * launch after it.  Results are identical either way.                      */
#define APUS_COMMIT_NC        0x10u
/* The statistics of this call replace the context's accumulated ones, as if
 * apus_stats_reset had run on the stream just before it (one launch fewer
 * per batch).                                                               */
#define APUS_COMMIT_STATS_FRESH 0x20u
/* a6's input from the same pass: the last NC determinant's (idx, term), else
 * the entry at log_get_tail's offset, else (0, 0) (apus_last_idx_term_batch).
 * With APUS_COMMIT_CHECKSUM on the segment kernel (APUS_BATCH_SHORT_WALKS) the
 * walk reads the last determinant's (idx, term) from the window it already
 * holds (an index below 2^32 and a term below 2^16; any other value, a ghost
 * case the walk cannot settle, or a deferred group is walked by the tail
 * launch), so no second pass over the ring is made; on the other walk kernels
 * the tail launch walks the determinants itself.  Results are identical
 * either way.                                                               */
#define APUS_COMMIT_LAST_IT   0x40u
/* The failover pass in the same tail launch (one read of each group's state
 * row and replica columns instead of one per call): the vote tally (a5, needs
 * b->vote_ack; outputs out->vote) and the vote-request ranking (a6, needs
 * b->sid, hb, vote_req and the local (idx, term); outputs out->rank).
 * Results are identical to apus_vote_batch / apus_vote_rank_batch on the same
 * batch (their inputs are not written by the commit call).                  */
#define APUS_COMMIT_VOTE      0x80u
#define APUS_COMMIT_RANK      0x100u
/* The lazy remote-commit publish (out->publish, out->ssn; needs remote_end,
 * remote_commit, lr_step, fail_count; b->rc_connected optional) in the same
 * tail launch: the tail walks the groups the walk kernel deferred in the lane
 * that finishes the group (the walk's new commit feeds it), so a walking call
 * must then supply out->new_commit.  force_log_pruning (out->force; needs
 * apply_offsets, ring, sid) in the tail of a call that does not walk.      */
#define APUS_COMMIT_PUBLISH     0x200u
#define APUS_COMMIT_FORCE_PRUNE 0x400u

typedef struct apus_prune_out {
    uint64_t *new_head;     /* [G] head after pruning (dare_server.c:2026-2058) */
    uint8_t  *append_head;  /* [G] 1 = leader appends a HEAD entry             */
    uint64_t *min_apply;    /* [G] min apply offset (before the HEAD test)     */
} apus_prune_out_t;

/* NC determinants of each follower for (idx, term) validation (a8).
 * dets: [G][n_followers][max_dets] apus_entry_det_t; det_len: [G][n_followers]
 * follower: [G][n_followers] server index (for the remote_commit fallback). */
typedef struct apus_nc_batch {
    uint32_t n_followers;
    uint32_t max_dets;          /* <= APUS_MAX_NC_ENTRIES                    */
    apus_entry_det_t *dets;
    uint32_t         *det_len;
    uint8_t          *follower;
    /* Optional (NULL = none): the leader's own NC determinants of [commit,
     * end) as apus_nc_build_batch / APUS_COMMIT_NC wrote them, [G][leader_max]
     * and leader_len [G].  A follower determinant k whose offset equals the
     * leader's k-th is checked against that determinant's (idx, term) -- the
     * entry the leader's log holds there -- instead of a gather of the
     * leader's header from the ring.  Same results; the leader's (idx, term)
     * then stream in coalesced rows.                                         */
    const apus_entry_det_t *leader_dets;
    const uint32_t         *leader_len;
    uint32_t leader_max;
    uint32_t pad;
} apus_nc_batch_t;

/* Per-batch aggregate statistics (device, uint64[APUS_STAT_COUNT]). */
#define APUS_STAT_DECISIONS       0   /* groups decided                       */
#define APUS_STAT_COMMITTED       1   /* entries committed                    */
#define APUS_STAT_ADVANCED        2   /* groups whose commit advanced         */
#define APUS_STAT_VOTES_WON       3
#define APUS_STAT_MISMATCHES      4   /* validation: followers whose end moved
                                         before their last NC entry           */
#define APUS_STAT_CORRUPT         5   /* walks stopped by the step guard      */
#define APUS_STAT_MIN_WATERMARK   6   /* min over groups of abs_base+new_head */
#define APUS_STAT_SLOW            7   /* commit groups the wave kernel handed to
                                         its exact one-lane walk (malformed or
                                         host-mapped rings, rings >= 2 GiB)   */
#define APUS_STAT_APPEND_SLOW     8   /* append groups the four-per-wave kernel
                                         handed to the per-group one          */
#define APUS_STAT_COUNT           9

/* ------------------------------------------------------------------------ */
/* Context                                                                   */
/* ------------------------------------------------------------------------ */
typedef struct apus_ctx apus_ctx_t;
typedef void *apus_stream_t;        /* hipStream_t (NULL = default stream)   */

const char *apus_version(void);
/* The layout revision of the structs in this header: a caller checks
 * apus_abi_version() == APUS_ABI_VERSION before passing any of them (the
 * library reads apus_batch_t / apus_commit_out_t fields of this revision).
 * 5: apus_batch_t.rc_connected; apus_commit_out_t.publish / ssn / force.
 * 6: apus_batch_t.vote_sit (168 B).
 * 7: apus_win_io_t / apus_vote_win_batch; APUS_FORCE_REFUSED;
 *    apus_commit_mark_tail.                                                */
#define APUS_ABI_VERSION 7
int apus_abi_version(void);
void apus_set_log(FILE *fp);        /* error sink; NULL = silent             */
/* A context may be used from up to 16 streams at once: each stream gets its
 * own launch scratch (per-block partial statistics, the deferred-walk list),
 * so batched calls on different streams run concurrently.  A launch on a
 * 17th stream waits for the device to drain and takes over the scratch of
 * the least recently used stream, so any number of streams may be used in
 * turn.  The statistics array is shared: concurrent batches accumulate into
 * it.                                                                       */
int  apus_ctx_create(int device, apus_ctx_t **out);
int  apus_ctx_destroy(apus_ctx_t *ctx);
/* device uint64[APUS_STAT_COUNT]; zeroed by apus_stats_reset */
uint64_t *apus_ctx_stats(apus_ctx_t *ctx);
int  apus_stats_reset(apus_ctx_t *ctx, apus_stream_t stream);
/* device->host copy of the stats (synchronises the stream) */
int  apus_stats_read(apus_ctx_t *ctx, uint64_t out[APUS_STAT_COUNT],
                     apus_stream_t stream);

/* ------------------------------------------------------------------------ */
/* Batched entry points (stream-ordered, asynchronous)                       */
/* ------------------------------------------------------------------------ */

/* a3 + a12 + a4: APUS reply-count commit walk, optional Adler-32 over the
 * walked entries, optional DARE median quorum.
 * Reference: update_remote_logs(), src/dare/dare_ibv_rc.c:1650-1758.       */
int apus_commit_batch(apus_ctx_t *ctx, const apus_batch_t *b,
                      const apus_commit_out_t *out, uint32_t flags,
                      apus_stream_t stream);
/* Measurement hook: the next apus_commit_batch call on this context launches
 * its walk kernel with `start` / `stop` (hipEvent_t, created by the caller)
 * as the kernel's own start and end timestamps (hipExtLaunchKernel: no marker
 * packets in the stream), so the walk's duration can be read with
 * hipEventElapsedTime while the call also runs its tail.  Consumed by that
 * call; NULL / NULL clears a pending pair.                                  */
int apus_commit_mark_walk(apus_ctx_t *ctx, void *start, void *stop);
/* The same for the call's tail kernel (quorum_tail_kernel: the deferred
 * walks, median, pruning, publish, failover pass and the statistics fold;
 * with APUS_BATCH_TAIL_ROWS its list launch).                              */
int apus_commit_mark_tail(apus_ctx_t *ctx, void *start, void *stop);

/* Which walk kernel apus_commit_batch would launch for this batch and these
 * flags (for measurement labels; no launch): info[0] 0 = commit_lane_kernel,
 * 1 = commit_wave_kernel, 2 = commit_seg_kernel; info[1] the hop walk
 * (APUS_BATCH_VAR_LEN); info[2] 64-group blocks handed out by a counter
 * (large batches); info[3] the persistent grid; info[4] the walk writes the NC
 * determinants; info[5] it records the last determinants' offsets.        */
int apus_commit_walk_info(apus_ctx_t *ctx, const apus_batch_t *b, uint32_t flags,
                          uint32_t info[6]);

/* a5: candidate-side vote tally, src/dare/dare_server.c:1327-1373.          */
int apus_vote_batch(apus_ctx_t *ctx, const apus_batch_t *b,
                    const apus_vote_out_t *out, apus_stream_t stream);

/* a6: voter-side request ranking / up-to-date test,
 * src/dare/dare_server.c:1526-1655 (needs b->sid, hb, vote_req,
 * last_idx_term).                                                           */
int apus_vote_rank_batch(apus_ctx_t *ctx, const apus_batch_t *b,
                         const apus_rank_out_t *out, apus_stream_t stream);

/* local last (idx, term) of every group as poll_vote_requests derives it
 * (dare_server.c:1598-1620: last NC determinant, else the tail entry);
 * out: device [G][2].  Feeds apus_batch_t.last_idx_term.                   */
int apus_last_idx_term_batch(apus_ctx_t *ctx, const apus_batch_t *b,
                             uint64_t *out, apus_stream_t stream);

/* a7: minimum applied offset for log pruning, dare_server.c:2026-2058
 * (+ log_get_tail, dare_log.h:402-457).  Also folds
 * min(abs_base + new_head) into APUS_STAT_MIN_WATERMARK when abs_base set.  */
int apus_prune_batch(apus_ctx_t *ctx, const apus_batch_t *b,
                     const apus_prune_out_t *out, apus_stream_t stream);

/* a8: (idx, term) validation, log_find_remote_end_offset,
 * dare_log.h:367-394, with the caller's empty-buffer rule
 * (dare_ibv_rc.c:1378-1384: end = log_offsets[i].commit).
 * remote_end_out: device [G][n_followers].  n_followers <= 13, dets 8-B
 * aligned.  Deviations (the reference reads undefined memory): det_len above
 * max_dets reads max_dets determinants; an empty buffer whose follower index
 * is not below n_replicas yields 0.                                         */
int apus_validate_batch(apus_ctx_t *ctx, const apus_batch_t *b,
                        const apus_nc_batch_t *nc, uint64_t *remote_end_out,
                        apus_stream_t stream);

/* a9: log_entries_to_nc_buf, dare_log.h:339-359: determinants of every entry
 * from commit to end (at most max_dets).  out dets [G][max_dets], len [G]. */
int apus_nc_build_batch(apus_ctx_t *ctx, const apus_batch_t *b,
                        apus_entry_det_t *dets, uint32_t max_dets,
                        uint32_t *len, apus_stream_t stream);

/* ---- log append + ack production ------------------------ */

/* One message to append: the tailq_entry_t fields get_tailq_message hands to
 * log_append_entry (dare_ibv_ud.c:780-790, dare_log.h:466-558).  `data_off`
 * locates the entry's `data` argument in apus_append_in_t.payload: an
 * sm_cmd_t {uint16_t len; uint8_t cmd[len]} for CSM-class types, a
 * dare_cid_t (16 B) for CONFIG, a uint64_t head for HEAD, unused for NOOP. */
typedef struct apus_append_entry {
    uint64_t req_id;
    uint64_t data_off;
    uint16_t clt_id;
    uint8_t  type;
    uint8_t  pad[5];
} apus_append_entry_t;                 /* 24 B */

typedef struct apus_append_in {
    const apus_append_entry_t *entries; /* [G][max_entries], in queue order   */
    const uint32_t *n_entries;          /* [G] messages per group (<= max);
                                           NULL = max_entries for every group */
    const uint64_t *term;               /* [G] term; NULL = SID_GET_TERM(sid[g])
                                           (dare_server.h:60, b->sid needed)  */
    const uint8_t  *payload;            /* device arena the data_off index    */
    uint64_t        payload_bytes;
    uint32_t        max_entries;
    uint32_t        flags;              /* APUS_APPEND_*; 0 = default         */
} apus_append_in_t;

/* apus_append_in_t.flags: append one group per wave even when max_entries
 * <= 16 (the default then places four groups per wave, one per 16-lane
 * segment, and hands any group whose batch is not one straight run back to
 * the per-group path).  Results are identical either way; the flag exists to
 * cross-check the two kernels. */
#define APUS_APPEND_PER_GROUP 0x1u

typedef struct apus_append_out {
    uint64_t *idx;       /* [G][max_entries] log_append_entry's return value:
                            the new entry's index, 0 when the log was full   */
    uint64_t *last_idx;  /* [G] last_write_csm_idx after the group's batch
                            (the last return value; unchanged input when the
                            group appended nothing).  NULL = not wanted.      */
} apus_append_out_t;

/* Appends every group's queued messages in order with log_append_entry's
 * exact semantics (index from the tail entry, log_get_tail when tail == len,
 * header wrap to 0, ghost header + rewrite at 0 when a command does not fit,
 * full log -> 0, prev_log_entry_head cleared by non-HEAD types).  state
 * (end, tail), ring and prev_head are updated in place.  A message whose
 * entry can never fit the ring (64 + cmd.len > len) or whose data lies
 * outside the payload arena -- out-of-bounds writes/reads in the reference --
 * stops that group: it and the group's remaining messages get idx 0 and
 * APUS_STAT_CORRUPT is incremented.                                         */
int apus_append_batch(apus_ctx_t *ctx, const apus_batch_t *b,
                      const apus_append_in_t *in, const apus_append_out_t *out,
                      apus_stream_t stream);

/* persist_new_entries (dare_server.c:1792-1810) for every replica copy of
 * every group.  All copies of a group's log are byte-identical (RDMA
 * replication), so the leader's ring stands for each of them.  Replica i
 * walks from its cursor old_end[g][i] while log_is_offset_larger(end,
 * old_end), following log_get_entry / log_fit_entry (ghost headers are
 * skipped), and for each entry:
 *   i == self_idx[g] (the leader): entry->sender = i   (IS_LEADER branch)
 *   i != self_idx[g] (a follower): entry->reply[i] = 1 (rc_send_entries_reply,
 *                                  dare_ibv_rc.c:1828-1863, writes that byte
 *                                  of the leader's entry)
 * limit[g][i] (NULL = no limit) caps the entries replica i persists in this
 * call -- the straggler model of the ack traces.  old_end is updated in
 * place.  Each cursor must lie on the log's entry chain, as the reference
 * keeps it (an entry boundary, or len on a log whose chain starts at 0): the
 * copies then walk the same chain and only write bytes (sender, reply[])
 * no walk reads.  A cursor off the chain walks misaligned headers whose
 * writes other copies may observe in any order (each reference copy would
 * see only its own).  A walk longer than len/64 + 4 steps (a corrupt ring; the
 * reference would not terminate) stops and counts APUS_STAT_CORRUPT.        */
typedef struct apus_persist_in {
    uint64_t       *old_end;   /* [G][R] in/out: dare_log_t.old_end of copy i */
    const uint32_t *limit;     /* [G][R] or NULL                              */
} apus_persist_in_t;

int apus_persist_batch(apus_ctx_t *ctx, const apus_batch_t *b,
                       const apus_persist_in_t *in, apus_stream_t stream);

/* ---- the proxy's stable-storage records, the BDB record format (8f.3) --
 * persist_new_entries (dare_server.c:1792-1810) hands every persisted entry
 * to proxy_store_cmd(&entry->clt_id) = stablestorage_save_request
 * (src/proxy/proxy.c:269-291), which reads the bytes from entry+24 as a
 * proxy message (src/include/proxy/proxy.h: proxy_msg_header {u16
 * connection_id; u8 action} = clt_id@24, type@26) and appends one record to
 * the server's Berkeley DB (RECNO, DB_APPEND, src/db/db-interface.c:65-95):
 *   CONNECT (4), CLOSE (6): PROXY_CONNECT_MSG_SIZE = PROXY_CLOSE_MSG_SIZE = 4 B
 *   SEND (5): PROXY_SEND_MSG_SIZE = 24 + data.cmd.len B, data at +8 of the
 *             message, so cmd.len is the u16 at entry+32 (reply[4..5] of the
 *             log entry -- the proxy message and the log entry disagree on the
 *             data offset; the record is what the reference stores)
 *   any other type: no record.
 * dump_records (db-interface.c:98-129) concatenates the records in recno
 * order: the snapshot (dare_server.c:618-640) that a recovering server loads
 * with stablestorage_load_records (proxy.c:306-336): from offset 0 while
 * len < size, SEND advances 24 + cmd.len (u16 at +8) and replays
 * do_action_send(connection_id, cmd.len, bytes at +10); CONNECT and CLOSE
 * advance 4 and replay do_action_connect / do_action_close.               */
#define APUS_REC_CONNECT_BYTES 4u     /* sizeof(proxy_connect_msg)            */
#define APUS_REC_SEND_BYTES 24u       /* sizeof(proxy_send_msg) (+ cmd.len)   */
#define APUS_REC_DATA_OFF 8u          /* offsetof(proxy_send_msg, data)       */

/* Records of the entries [cursor, end) of every group's log, appended to the
 * group's record dump -- the store side (persist_new_entries' walk, the
 * entry bytes as they are when the call runs; the ring is not modified).
 * cursor[g] is the server's old_end (in/out).  A record that would run past
 * the ring's len (the reference reads past its log) or past cap stops the
 * group there (cursor at that entry) and counts APUS_STAT_CORRUPT.  cap must
 * fit the uint32_t records_len (db-interface.c:21).                        */
typedef struct apus_records_io {
    uint64_t *cursor;      /* [G] in/out: where the persist walk starts      */
    uint8_t  *dump;        /* [G][cap] each group's records, recno order     */
    uint64_t  cap;         /* bytes per group dump                           */
    uint32_t *dump_len;    /* [G] in/out: records_len                        */
    uint32_t *n_records;   /* [G] out: records appended by this call (or NULL)*/
} apus_records_io_t;

/* Kernels: 16 lanes per group confirm up to 16 entries per step when the
 * entry lengths repeat (a log of equal-size commands); with b->flags &
 * APUS_BATCH_LANE_IMPL one lane per group follows the chain.  Same results. */
int apus_records_store_batch(apus_ctx_t *ctx, const apus_batch_t *b,
                             const apus_records_io_t *io, apus_stream_t stream);

/* One replayed record of a snapshot (stablestorage_load_records).           */
typedef struct apus_record_ref {
    uint32_t offset;        /* of the record in its dump                     */
    uint32_t data_len;      /* SEND: cmd.len (bytes at offset + 10); else 0  */
    uint16_t connection_id;
    uint8_t  action;        /* 4 CONNECT, 5 SEND, 6 CLOSE                    */
    uint8_t  pad[5];
} apus_record_ref_t;        /* 16 B */

/* stablestorage_load_records over n snapshots (dump k at dump + k*stride,
 * size[k] bytes): the replay plan of each (at most max_plan records kept,
 * all counted), counts[k][0..2] = CONNECT / SEND / CLOSE records, status[k]:
 * 0 every byte consumed; 1 an unknown action at the stop offset (the
 * reference never leaves its loop: len does not advance); 2 the last record
 * runs past size (the reference reads past the buffer): not replayed.  A
 * size above stride is taken as stride (the walk never reads another dump). */
typedef struct apus_records_load_io {
    const uint8_t     *dump;
    uint64_t           stride;
    const uint32_t    *size;      /* [n] */
    uint64_t           n;
    apus_record_ref_t *plan;      /* [n][max_plan] or NULL */
    uint32_t           max_plan;
    uint32_t           flags;     /* APUS_BATCH_LANE_IMPL: one lane per snapshot
                                     instead of 16-lane speculative segments
                                     (cross-checking); same results          */
    uint32_t          *n_records; /* [n] */
    uint32_t          *counts;    /* [n][3] or NULL */
    uint32_t          *status;    /* [n] */
    uint32_t          *stop;      /* [n] offset where the walk ended, or NULL */
} apus_records_load_io_t;

int apus_records_load_batch(apus_ctx_t *ctx, const apus_records_load_io_t *io, apus_stream_t stream);

/* ---- apply / config scan --------------------------------- */

/* poll_config_entries, src/dare/dare_server.c:2133-2187, with update_cid
 * (:2193-2226) and equal_cid (src/include/dare/dare_config.h:48-56): every
 * group walks its log from data.config.cid_offset to end.  A CONFIG entry
 * with idx > cid_idx whose cid differs from state.cid replaces it (in place)
 * and records the entry's req_id / clt_id; a HEAD entry at or before commit
 * moves the head candidate; state.head advances to it when circularly
 * larger.  cid_offset ends at the walk's offset, or commit when that is
 * larger.  departed[g] gets bit i for every server update_cid disconnects
 * (dare_ib_disconnect_server; bit self = "somebody removed me", the caller
 * shuts down).  A walk longer than len/64 + 4 steps stops (APUS_STAT_CORRUPT;
 * the reference would not terminate) with the group's outputs as they were. */
typedef struct apus_config_io {
    uint64_t       *cid_offset; /* [G] in/out data.config.cid_offset           */
    const uint64_t *cid_idx;    /* [G] data.config.cid_idx                     */
    uint64_t       *req_id;     /* [G] in/out data.config.req_id               */
    uint16_t       *clt_id;     /* [G] in/out data.config.clt_id               */
    uint16_t       *departed;   /* [G] out, or NULL                            */
} apus_config_io_t;

int apus_config_scan_batch(apus_ctx_t *ctx, const apus_batch_t *b,
                           const apus_config_io_t *io, apus_stream_t stream);

/* apply_committed_entries, src/dare/dare_server.c:1815-1974: every group
 * walks [apply, commit) (log_get_entry / log_fit_entry; state.apply updated
 * in place).  IS_LEADER = SID_GET_L(sid) && SID_GET_IDX(sid) == self_idx
 * (dare_server.c:46-48).  Client (CSM-class) entries are applied: the state
 * machine call itself (proxy_do_action / proxy_update_state) belongs to the
 * host, which gets the count and the range [apply_in, apply_out); each one
 * sets last_applied = (idx, term, offset + len) and last_csm_idx = idx.  On
 * the leader an unstable CONFIG entry of the current epoch moves state.cid
 * EXTENDED -> TRANSIT or TRANSIT -> STABLE (servers size[1]..size[0]-1
 * removed: departed bits, APUS_EV_SELF_REMOVED for self) and requests the
 * CONFIG re-append of log_append_entry(term, req_id, clt_id, CONFIG, &cid):
 * the request is written to cfg_entries / cfg_payload in apus_append_batch's
 * input format (data_off indexes cfg_payload), so appending them in order
 * with apus_append_batch completes the reference's step (the appended
 * entries lie past commit, so the scan never reads them).  A group with more
 * than max_cfg such entries stops before the next one (apply stays there;
 * APUS_EV_CFG_FULL) and resumes on the next call.  Followers apply every
 * entry type's bookkeeping the same way as the reference (only CSM entries
 * touch last_applied).                                                      */
#define APUS_EV_CFG_REPLY      1   /* a STABLE CONFIG with req_id != 0: client reply */
#define APUS_EV_JOIN_REPLY     2   /* EXTENDED -> TRANSIT with req_id != 0: reply to the joining server */
#define APUS_EV_SELF_REMOVED   4   /* DIE_AF_COMMIT: the leader removed itself */
#define APUS_EV_CFG_FULL       8   /* stopped at max_cfg CONFIG re-appends     */
typedef struct apus_apply_io {
    uint64_t            *req_id;       /* [G] in/out data.config.req_id             */
    uint16_t            *clt_id;       /* [G] in/out data.config.clt_id             */
    uint64_t            *last_applied; /* [G][3] in/out last_applied_entry (idx, term, offset) */
    uint64_t            *last_csm_idx; /* [G] in/out data.last_cmt_write_csm_idx    */
    uint32_t            *n_applied;    /* [G] out: client entries applied, or NULL  */
    uint16_t            *departed;     /* [G] out, or NULL                          */
    uint8_t             *events;       /* [G] out APUS_EV_*, or NULL                */
    apus_append_entry_t *cfg_entries;  /* [G][max_cfg] out                          */
    uint8_t             *cfg_payload;  /* [G][max_cfg][16] out: the appended dare_cid_t */
    uint32_t            *n_cfg;        /* [G] out                                   */
    uint32_t             max_cfg;
    uint32_t             pad;
} apus_apply_io_t;

int apus_apply_batch(apus_ctx_t *ctx, const apus_batch_t *b,
                     const apus_apply_io_t *io, apus_stream_t stream);

/* ---- the election-win transition (BASELINE config 5's reconfiguration) --
 * The rest of poll_vote_count after the tally (src/dare/dare_server.c:
 * 1355-1362, 1389-1510), for every group polling() asks to count votes:
 * IS_CANDIDATE (dare_server.c:49-51,1110-1112: SID_GET_IDX(sid) == self_idx,
 * the L bit clear, SID_GET_TERM(sid) != 0).  Other groups are not touched
 * (APUS_WIN_NOT_CANDIDATE).  The tally itself is a5 (apus_vote_batch, or
 * APUS_COMMIT_VOTE on this batch): io->won / voters / new_commit are its
 * outputs.  A candidate, in the reference's order:
 *   1. the tally's side effects (:1355-1362): remote_commit[i] = vote_ack[i],
 *      lr_step[i] = LR_GET_NCE_LEN for every voter i; state.commit =
 *      new_commit.  Lost: APUS_WIN_LOST, nothing more.  Won:
 *   2. server_update_sid (:1389-1395, :2288-2297): sid |= L by a
 *      compare-and-swap on the value read;
 *   3. poll_config_entries (:2133-2187) from io->cid_offset (as
 *      apus_config_scan_batch);
 *   4. apply_committed_entries (:1815-1974) as the leader (as
 *      apus_apply_batch), the CONFIG re-appends appended to the log in place
 *      when they are met, as the reference appends them (io->n_cfg);
 *   5. the blank entry (:1411-1491), log_append_entry (dare_log.h:466-558) at
 *      SID_GET_TERM(sid):
 *        STABLE: req_id = clt_id = 0, a CONFIG entry          APUS_WIN_CONFIG
 *        else a scan from cid_offset: a CONFIG entry with idx > cid_idx ->
 *        a NOOP                                                APUS_WIN_NOOP
 *        else, on the last entry the scan examined, data.cid.state ==
 *        CID_EXTENDED -> state TRANSIT                         APUS_WIN_TRANSIT
 *        otherwise state STABLE, servers size[0]-1 down to size[1]+1 removed
 *        (departed bits; self: APUS_EV_SELF_REMOVED), size[0] = size[1],
 *        size[1] = 0                                           APUS_WIN_STABLE
 *        and then a CONFIG entry with the config's req_id / clt_id;
 *      last_write_csm_idx = the append's return (0: the log was full);
 *   6. become_leader (:1504-1508): apply_offsets[i] = head for
 *      i < get_extended_group_size (columns past n_replicas do not exist).
 * The host keeps what the reference does beyond the log: the heartbeat and
 * pruning timers, ep_dp_reset_wait_idx, the log access (:1494-1517), the
 * client replies of events and the disconnects of departed.
 * Deviations (undefined in the reference): the unstable branch with no entry
 * examined (cid_offset at end) reads an uninitialised pointer (:1456): no
 * blank entry, step 6 runs (APUS_WIN_UNDEFINED).  A walk longer than
 * len/64 + 4 steps or offsets the batched append refuses stop the group where
 * they are met, with its updates up to there (APUS_WIN_CORRUPT,
 * APUS_STAT_CORRUPT); so does a failed compare-and-swap (another writer
 * changed the SID; the reference exits).                                    */
#define APUS_WIN_NOT_CANDIDATE 0
#define APUS_WIN_LOST          1
#define APUS_WIN_CONFIG        2
#define APUS_WIN_NOOP          3
#define APUS_WIN_TRANSIT       4
#define APUS_WIN_STABLE        5
#define APUS_WIN_UNDEFINED     6
#define APUS_WIN_CORRUPT       7
typedef struct apus_win_io {
    const uint8_t  *won;                /* [G] the tally's outputs (apus_vote_out_t) */
    const uint16_t *voters;             /* [G]                                       */
    const uint64_t *new_commit;         /* [G]                                       */
    uint64_t       *cid_offset;         /* [G] in/out data.config.cid_offset         */
    const uint64_t *cid_idx;            /* [G] data.config.cid_idx                   */
    uint64_t       *req_id;             /* [G] in/out data.config.req_id             */
    uint16_t       *clt_id;             /* [G] in/out data.config.clt_id             */
    uint64_t       *last_applied;       /* [G][3] in/out last_applied_entry          */
    uint64_t       *last_csm_idx;       /* [G] in/out data.last_cmt_write_csm_idx    */
    uint64_t       *last_write_csm_idx; /* [G] in/out data.last_write_csm_idx        */
    uint8_t        *outcome;            /* [G] out APUS_WIN_*                         */
    uint8_t        *events;             /* [G] out APUS_EV_* (apply, removal), or NULL */
    uint16_t       *departed;           /* [G] out: servers disconnected by the scan,
                                           the apply and the blank entry, or NULL   */
    uint32_t       *n_applied;          /* [G] out: client entries applied, or NULL  */
    uint32_t       *n_cfg;              /* [G] out: CONFIG re-appends, or NULL       */
} apus_win_io_t;

/* needs b->ring, state (or images + cid), self_idx, sid, vote_ack,
 * remote_commit, lr_step, apply_offsets; b->prev_head optional (the appends
 * clear it, dare_log.h:477-480) */
int apus_vote_win_batch(apus_ctx_t *ctx, const apus_batch_t *b,
                        const apus_win_io_t *io, apus_stream_t stream);

/* ---- log replication step machine ----------------------- */

/* Completion status of the log-replication WR of (group g, server i), as
 * handle_lr_work_completion receives it (dare_ibv_rc.c:3126-3196). */
#define APUS_WC_NONE     0   /* no completion for (g, i) in this call          */
#define APUS_WC_SUCCESS  1   /* wc_rc == WC_SUCCESS                            */
#define APUS_WC_FAILED   2   /* any other wc_rc                                */
#define APUS_WC_STALE    3   /* wr_id != servers[i].next_wr_id (an old SSN):
                                ignored, dare_ibv_rc.c:3136                    */

/* The work request log_adjustment posts for (g, i) (dare_ibv_rc.c:1347-1441):
 * the caller posts it (RDMA is the host's) after the call. */
#define APUS_LR_POST_NONE         0
#define APUS_LR_POST_READ_NC_LEN  1  /* RDMA READ remote nc_buf[self].len into
                                        log->nc_buf[i].len (LR_GET_NCE_LEN)    */
#define APUS_LR_POST_READ_NC      2  /* RDMA READ nc_buf[self].entries, nc_len*24
                                        bytes, into log->nc_buf[i] (LR_GET_NCE) */
#define APUS_LR_POST_WRITE_END    3  /* RDMA WRITE log_offsets[i].end to the
                                        remote log->end (LR_SET_END)           */

/* Per-server replication state the step machine reads and writes.  Every
 * [G][R] array is row-major by server index, as in apus_batch_t.  The batch
 * supplies state (commit updated in place), self_idx, fail_count, lr_step
 * (in/out), vote_ack, remote_commit (in/out, log_offsets[i].commit) and
 * remote_end (in/out, log_offsets[i].end). */
typedef struct apus_lr_io {
    uint8_t                *send_flag;    /* [G][R] in/out servers[i].send_flag   */
    uint8_t                *send_count;   /* [G][R] in/out servers[i].send_count
                                             (completion only)                   */
    const uint8_t          *wc;           /* [G][R] APUS_WC_* (completion only)  */
    const uint16_t         *rc_connected; /* [G] bit i = servers[i].ep->rc_connected
                                             (adjust only; NULL = all connected) */
    const uint64_t         *nc_len;       /* [G][R] log->nc_buf[i].len (adjust)  */
    const apus_entry_det_t *nc_dets;      /* [G][R][max_dets] log->nc_buf[i].entries
                                             (adjust; read at LR_SET_END only)   */
    uint64_t               *ssn;          /* [G] in/out the leader's ssn (adjust) */
    uint8_t                *post;         /* [G][R] out APUS_LR_POST_* (adjust)  */
    uint32_t                max_dets;     /* <= APUS_MAX_NC_ENTRIES              */
    uint32_t                pad;
} apus_lr_io_t;

/* handle_lr_work_completion (dare_ibv_rc.c:3126-3196) for every (g, i) with
 * wc != APUS_WC_NONE, one thread per pair: success advances next_lr_step
 * (LR_UPDATE_LOG: by send_count 0/1/2; LR_UPDATE_END -> LR_UPDATE_LOG; other
 * steps ++, uint8 arithmetic) and re-arms send_flag; failure re-arms
 * send_flag (LR_UPDATE_LOG with send_count 2: send_count = 0 instead).      */
int apus_lr_completion_batch(apus_ctx_t *ctx, const apus_batch_t *b,
                             const apus_lr_io_t *io, apus_stream_t stream);

/* log_adjustment (dare_ibv_rc.c:1292-1451), the leader's per-server log
 * adjustment, for every group (lane per group, servers in index order as the
 * reference loops).  Servers are skipped when they are self or OFF in cid,
 * fail_count >= PERMANENT_FAILURE, send_flag == 0, not rc_connected, or
 * vote_ack[i] == len.  The first non-skipped server whose step is below
 * LR_UPDATE_LOG increments ssn[g].  LR_GET_WRITE: remote_commit[i] =
 * vote_ack[i], step LR_GET_NCE_LEN, falling through to LR_GET_NCE_LEN: the
 * leader's commit becomes vote_ack[i] when circularly larger
 * (log_is_offset_larger), post READ_NC_LEN.  LR_GET_NCE: nc_len 0 -> remote
 * end = remote_commit, step LR_UPDATE_LOG, nothing posted; else post
 * READ_NC.  LR_SET_END: remote_end[i] = log_find_remote_end_offset over
 * nc_dets[g][i][0..nc_len) (dare_log.h:367-394), post WRITE_END.  A posting
 * server gets send_flag = 0.  post[g][i] is written for every i < R.
 * Deviations (the reference reads undefined memory): an LR_SET_END buffer
 * with nc_len 0 yields remote_commit[i] (the caller's rule for an empty
 * buffer, as apus_validate_batch); nc_len above max_dets is read as max_dets;
 * servers i >= n_replicas are never visited.                                */
int apus_log_adjust_batch(apus_ctx_t *ctx, const apus_batch_t *b,
                          const apus_lr_io_t *io, apus_stream_t stream);

/* Synthetic trace generator (device): fills ring/state/per-replica arrays
 * of b exactly as oracle/apus_oracle.c's apus_oracle_gen_group does.        */
typedef struct apus_gen_cfg {
    uint64_t seed;
    uint64_t gid_base;          /* global id of group 0 of this batch (shard) */
    uint32_t n_entries;         /* E: entries in the not-committed batch      */
    uint32_t n_history;         /* committed entries before the batch         */
    uint32_t len_min, len_max;  /* cmd.len range for CSM-class entries        */
    uint32_t ring_len;          /* dare_log_t.len of every group              */
    uint32_t p_full_ack;        /* P(follower acked all E) in 1/65536         */
    uint32_t straggler;         /* 1: one follower acks only U[0, E/4]        */
    uint32_t type_mix;          /* 0: all SEND(5); 1: mixed NOOP/CONFIG/HEAD/
                                   CONNECT/SEND/CLOSE                          */
    uint32_t cid_mix;           /* 0: STABLE size R; 1: 60% STABLE, 20%
                                   EXTENDED (R-1 -> R), 20% TRANSIT           */
    uint32_t garbage_reply;     /* P(an ack byte is 2 instead of 1) /65536    */
    uint32_t self_random;       /* 1: leader index random in [0,R)            */
    uint32_t p_vote_ack;        /* P(vote_ack present) in 1/65536             */
    uint32_t fill_garbage;      /* 1: pre-fill rings with random bytes        */
    uint32_t hist_len_max;      /* cmd.len bound of the n_history committed
                                   entries (0: len_max): rings sized for the
                                   batch, not for maximum-length history      */
} apus_gen_cfg_t;

int apus_gen_batch(apus_ctx_t *ctx, const apus_batch_t *b,
                   const apus_gen_cfg_t *cfg, apus_stream_t stream);

/* RCCL all-reduce of the stats over a communicator: SUM over
 * every statistic but APUS_STAT_MIN_WATERMARK, MIN over that one, issued as
 * one ncclGroupStart/End (a single fused launch).  comm is an ncclComm_t
 * created by the caller (e.g. via apus_comm_init_rank).                     */
int apus_comm_get_unique_id(char id_out[128]);
int apus_comm_init_rank(apus_ctx_t *ctx, int nranks, const char id[128],
                        int rank);
int apus_stats_allreduce(apus_ctx_t *ctx, apus_stream_t stream);
/* the same under the name SURVEY.md 8(b) lists for the batched boundary      */
int apus_allreduce_stats(apus_ctx_t *ctx, apus_stream_t stream);

/* ------------------------------------------------------------------------ */
/* Scalar drop-ins (reference-shaped structs, default context, device 0 or  */
/* APUS_DEVICE).  Each copies its inputs to device scratch, runs the batched */
/* kernel with G = 1 and returns synchronously.  Calls from several threads  */
/* are serialised on the default context (one at a time).                    */
/* ------------------------------------------------------------------------ */

/* Where a scalar call reads the ring.  The library never registers or maps
 * memory it did not allocate:
 *  - a log from apus_log_new is pinned, mapped host memory the library owns;
 *    the kernels read its ring in place (zero-copy), so remote writes into it
 *    (reply[], end) are seen by the next call as in the reference;
 *  - any other log is staged: the call copies the ring ranges the reference
 *    reads for it into the default context's own pinned image -- the chain
 *    [commit, end) for the walk and the NC build, plus [apply, end) and
 *    [head, end) when log_get_tail scans (tail == len), and the 64-B header
 *    at each determinant offset / the tail -- and the kernels read that.
 *    Every entry of a log built by log_append_entry lies in [head, end), so
 *    results are the reference's; a corrupt log whose entry chain leaves the
 *    staged ranges reads the poison byte 0xFF there (deterministic: the
 *    reference's result on a copy of the log with those bytes set to 0xFF;
 *    tests/test_gpu_parity.py::test_scalar_walk_malformed).
 *  The walk, median, vote tally, pruning minimum and publish run in ONE
 *  launch: the state, the columns and the staged ring bytes (up to 3 KB)
 *  travel in the kernel arguments, results come back through mapped pinned
 *  memory; a longer walk window takes the staged path above.              */

/* log_new (dare_log.h:120-137) for the scalar calls: allocates header + len
 * ring bytes (+64 B of tail pad) as pinned, mapped host memory, zeroed, with
 * len = end = tail = old_end = len.  Register it with the NIC as the
 * reference registers its log (ibv_reg_mr, dare_ibv_rc.c:240-276).          */
int apus_log_new(uint64_t len, apus_log_t **out);

/* log_free (dare_log.h:142-149) for a log from apus_log_new; waits for a
 * scalar call in flight.  APUS_INSUCCESS: not allocated by apus_log_new.   */
int apus_log_free(apus_log_t *log);

/* Scalar-call accounting: calls that read a log in place, calls that staged,
 * bytes staged, and logs currently allocated by apus_log_new.              */
int apus_scalar_path_stats(uint64_t *in_place_calls, uint64_t *staged_calls,
                           uint64_t *staged_bytes, uint32_t *owned_logs);

/* APUS commit rule (dare_ibv_rc.c:1725-1758). new_commit receives the commit
 * offset after the walk; *committed = 1 when it advanced (the caller then
 * sets log->commit = config->cid_offset = *new_commit).                     */
int apus_commit_reply_walk(const apus_log_t *log,
                           const apus_server_config_t *config,
                           uint64_t *new_commit, int *committed);

/* DARE median quorum (dare_ibv_rc.c:1650-1723); remote ends come from
 * ctrl->log_offsets[i].end, gates from config->servers[i].                  */
int apus_commit_median(const apus_log_t *log,
                       const apus_server_config_t *config,
                       const apus_ctrl_data_t *ctrl, uint64_t *median);

/* poll_vote_count tally (dare_server.c:1330-1373).  Returns 1 if won, 0 if
 * not, APUS_INSUCCESS on error; vc/new_commit/voters as in apus_vote_out_t. */
int apus_vote_tally(const apus_log_t *log,
                    const apus_server_config_t *config,
                    const apus_ctrl_data_t *ctrl, uint8_t vc[2],
                    uint64_t *new_commit, uint16_t *voters);

/* poll_vote_requests ranking (dare_server.c:1526-1655).  The local
 * (idx, term) is derived on the device from the log (NC buffer / tail).
 * Like the reference, requests that lose are cleared in ctrl->vote_req.     */
int apus_vote_rank(const apus_log_t *log,
                   const apus_server_config_t *config,
                   apus_ctrl_data_t *ctrl, uint8_t *outcome,
                   uint64_t *new_sid, apus_cid_t *new_cid, uint16_t *cleared);

/* log_pruning minimum (dare_server.c:2026-2058).  Like the reference, the
 * apply offsets of OFF servers are reset to log->apply in ctrl.            */
int apus_min_apply(const apus_log_t *log,
                   const apus_server_config_t *config,
                   apus_ctrl_data_t *ctrl, int prev_log_entry_head,
                   uint64_t *new_head, int *append_head);

/* The lazy remote-commit publish that ends update_remote_logs
 * (dare_ibv_rc.c:1760-1822), on log->commit as the caller left it after the
 * commit rule: for every server it visits, ctrl->log_offsets[i].commit is set
 * in place as the reference sets it; bit i of *post = the 8-B commit write the
 * caller posts to server i; *ssn is incremented when any is posted.
 * rc_connected: bit i = servers[i].ep->rc_connected.                        */
int apus_publish_commit(const apus_log_t *log, const apus_server_config_t *config,
                        apus_ctrl_data_t *ctrl, uint16_t rc_connected, uint64_t *ssn,
                        uint16_t *post);

/* force_log_pruning (dare_server.c:2069-2122).  On APUS_FORCE_REMOVE the log
 * (the CONFIG entry's bytes, end, tail), config->cid / req_id / clt_id,
 * ctrl->apply_offsets and *prev_log_entry_head are updated in place as the
 * reference updates them (dare_ib_disconnect_server(*target) is the caller's);
 * then, as for every outcome but APUS_FORCE_NONE, log_pruning's results:
 * *new_head / *append_head as apus_min_apply reports them (the HEAD append is
 * the caller's, as there).  Returns APUS_FORCE_* or APUS_INSUCCESS on error. */
int apus_force_log_pruning(apus_log_t *log, apus_server_config_t *config,
                           apus_ctrl_data_t *ctrl, int *prev_log_entry_head,
                           uint8_t *target, uint64_t *cfg_idx, uint64_t *new_head,
                           int *append_head);

/* log_find_remote_end_offset (dare_log.h:367-394).  nc->len == 0 is
 * undefined in the reference; this returns APUS_ERROR for it.              */
int apus_find_remote_end(const apus_log_t *log, const apus_nc_buf_t *nc,
                         uint64_t *remote_end);

/* log_adjustment (dare_ibv_rc.c:1292-1451) on the reference's structs:
 * reads config->servers[i] (fail_count, send_flag, next_lr_step, i <
 * config->len), ctrl->vote_ack and log->nc_buf[i]; updates log->commit,
 * servers[i].next_lr_step / send_flag, ctrl->log_offsets[i].commit / .end
 * and *ssn in place, as the reference does.  post[i] receives the
 * APUS_LR_POST_* work request the caller posts (post_send, :1428-1445).
 * rc_connected: bit i = servers[i].ep->rc_connected.  Same kernel and
 * deviations as apus_log_adjust_batch.                                      */
int apus_log_adjustment(apus_log_t *log, apus_server_config_t *config,
                        apus_ctrl_data_t *ctrl, uint16_t rc_connected,
                        uint64_t *ssn, uint8_t post[APUS_MAX_SERVER_COUNT]);

/* handle_lr_work_completion (dare_ibv_rc.c:3126-3196) for one server_t:
 * wc = APUS_WC_SUCCESS / APUS_WC_FAILED (APUS_WC_STALE / _NONE: unchanged). */
int apus_lr_work_completion(apus_server_t *server, int wc);

/* log_entries_to_nc_buf (dare_log.h:339-359). */
int apus_entries_to_nc_buf(const apus_log_t *log, apus_nc_buf_t *nc);

#ifdef __cplusplus
}
#endif
#endif /* APUS_GPU_H */
