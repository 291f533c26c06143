/*
 * dare_poll.c -- libapus_gpu from C, as the reference's DARE server would call it
 * (INTEGRATION.md section 2): one leader's dare_log_t and its server_config_t /
 * ctrl_data_t, laid out byte for byte as the reference lays them out, driven
 * through the scalar drop-ins in polling()'s order:
 *
 *   update_remote_logs   apus_commit_reply_walk  (dare_ibv_rc.c:1725-1758)
 *                        apus_commit_median      (:1650-1723)
 *                        apus_publish_commit     (:1760-1822, on the walk's commit)
 *   log_pruning          apus_min_apply          (dare_server.c:2026-2058)
 *   poll_vote_count      apus_vote_tally         (:1330-1373)
 *   log adjustment       apus_entries_to_nc_buf  (dare_log.h:339-359)
 *                        apus_find_remote_end    (dare_log.h:367-394)
 *
 * The log comes from apus_log_new (pinned, mapped host memory the GPU reads in
 * place -- the memory the reference would ibv_reg_mr).  Usage:
 *   dare_poll SEED DUMP_PATH
 * fills the log deterministically from SEED, writes the call inputs (the log
 * header + ring, config, servers, ctrl_data, the follower's NC buffer) to
 * DUMP_PATH before any call, and prints one JSON line of results; the GPU test
 * (tests/test_c_dropin.py) runs the reference's own code on the dump.
 */
#include <inttypes.h>
#include <stdio.h>
#include <stdlib.h>
#include <string.h>

#include "apus_gpu.h"

#define R 3
#define LEN 16384u
#define ELEN 128u

static uint64_t rng_state;
static uint64_t splitmix(void)
{
    uint64_t z = (rng_state += 0x9E3779B97F4A7C15ull);
    z = (z ^ (z >> 30)) * 0xBF58476D1CE4E5B9ull;
    z = (z ^ (z >> 27)) * 0x94D049BB133111EBull;
    return z ^ (z >> 31);
}

#define CHECK(x)                                                                 \
    do {                                                                         \
        int rc_ = (x);                                                           \
        if (rc_ != APUS_OK) {                                                    \
            fprintf(stderr, "%s failed: %d\n", #x, rc_);                         \
            return 1;                                                            \
        }                                                                        \
    } while (0)

int main(int argc, char **argv)
{
    if (argc < 3) {
        fprintf(stderr, "usage: %s SEED DUMP_PATH\n", argv[0]);
        return 2;
    }
    rng_state = strtoull(argv[1], NULL, 0);
    apus_set_log(stderr);

    /* ---- the leader's log: n entries of 128 B (64-B header + a 64-B SET),
     * starting anywhere on the ring (the batch may wrap: ghost header or a
     * header that does not fit, dare_log.h:316-332) ---- */
    apus_log_t *log = NULL;
    CHECK(apus_log_new(LEN, &log));
    const uint32_t n = 24 + (uint32_t)(splitmix() % 40);          /* entries written */
    const uint32_t hist = 4 + (uint32_t)(splitmix() % 8);          /* already committed */
    uint64_t off = 16u * (splitmix() % (LEN / 16));
    const uint64_t first = off;
    uint64_t ends[64], tail = 0;
    uint32_t acked[R];
    for (int i = 0; i < R; i++) acked[i] = hist + (uint32_t)(splitmix() % (n - hist + 1));
    acked[0] = n;                                                  /* the leader itself */
    for (uint32_t k = 0; k < n; k++) {
        if (LEN - off < APUS_ENTRY_HDR) off = 0;                   /* header does not fit: wrap */
        else if (LEN - off < ELEN) {                               /* a ghost header at off */
            apus_log_entry_t *g = (apus_log_entry_t *)(log->entries + off);
            memset(g, 0, sizeof *g);
            g->idx = 1000 + k;
            g->term = 7;
            g->type = 5;
            g->data.cmd.len = (uint16_t)(ELEN - APUS_ENTRY_HDR);
            off = 0;
        }
        apus_log_entry_t *e = (apus_log_entry_t *)(log->entries + off);
        e->idx = 1000 + k;
        e->term = 7;
        e->req_id = splitmix();
        e->clt_id = (uint16_t)splitmix();
        e->type = 5;                                               /* SEND (APUS CSM class) */
        e->data.cmd.len = (uint16_t)(ELEN - APUS_ENTRY_HDR);
        for (uint32_t b = 0; b < ELEN - APUS_ENTRY_HDR - 2; b++) log->entries[off + 50 + b] = (uint8_t)splitmix();
        for (int i = 1; i < R; i++) e->reply[i] = k < acked[i];   /* prefix-monotone acks */
        tail = off;
        off += ELEN;
        ends[k] = off;
    }
    log->len = LEN;
    log->end = off;
    log->tail = tail;
    log->commit = hist ? ends[hist - 1] : first;
    log->apply = first;
    log->head = first;
    log->old_end = log->end;
    log->old_commit = log->commit;

    /* ---- server_config_t (3 servers, STABLE, all on; self = 0) and ctrl_data_t ---- */
    apus_server_t servers[APUS_MAX_SERVER_COUNT];
    memset(servers, 0, sizeof servers);
    apus_server_config_t cfg;
    memset(&cfg, 0, sizeof cfg);
    cfg.cid.epoch = 1;
    cfg.cid.size[0] = R;
    cfg.cid.state = APUS_CID_STABLE;
    cfg.cid.bitmask = (1u << R) - 1u;
    cfg.servers = servers;
    cfg.idx = 0;
    cfg.len = R;
    static apus_ctrl_data_t ctrl;
    memset(&ctrl, 0, sizeof ctrl);
    for (int i = 0; i < R; i++) {
        servers[i].next_lr_step = APUS_LR_UPDATE_LOG;
        servers[i].fail_count = (uint8_t)(i == 2 && (splitmix() & 1));   /* one follower failing once */
        ctrl.log_offsets[i].end = acked[i] ? ends[acked[i] - 1] : first;
        ctrl.log_offsets[i].commit = hist ? ends[hist - 1] : first;
        ctrl.vote_ack[i] = (splitmix() & 3) ? ends[(hist + (uint32_t)(splitmix() % (n - hist))) % n] : log->len;
        ctrl.apply_offsets[i] = ends[(uint32_t)(splitmix() % hist)];
    }
    /* a follower's NC buffer: the leader's determinants, the term changed at m */
    static apus_nc_buf_t nc_lead, nc_fol;

    /* ---- the inputs, before any call writes to them ---- */
    FILE *f = fopen(argv[2], "wb");
    if (!f) {
        perror(argv[2]);
        return 1;
    }
    fwrite(log, 1, 64, f);                                         /* head .. len */
    fwrite(log->entries, 1, LEN, f);
    fwrite(&cfg, 1, sizeof cfg, f);
    fwrite(servers, 1, sizeof servers, f);
    fwrite(&ctrl, 1, sizeof ctrl, f);

    /* ---- polling(): the leader's commit path ---- */
    uint64_t new_commit = 0, median = 0, ssn = 0, new_head = 0, vcommit = 0, rend = 0;
    int committed = 0, append_head = 0;
    uint16_t post = 0, voters = 0;
    uint8_t vc[2] = { 0, 0 };
    CHECK(apus_commit_reply_walk(log, &cfg, &new_commit, &committed));
    CHECK(apus_commit_median(log, &cfg, &ctrl, &median));
    const uint64_t commit0 = log->commit;
    if (committed) log->commit = cfg.cid_offset = new_commit;    /* the caller's update (:1744-1757) */
    CHECK(apus_publish_commit(log, &cfg, &ctrl, 0xFFFF, &ssn, &post));
    uint64_t rcommit[R];
    for (int i = 0; i < R; i++) rcommit[i] = ctrl.log_offsets[i].commit;
    log->commit = commit0;                                         /* the other calls see the input log */
    CHECK(apus_min_apply(log, &cfg, &ctrl, 0, &new_head, &append_head));
    const int won = apus_vote_tally(log, &cfg, &ctrl, vc, &vcommit, &voters);
    if (won < 0) return 1;
    CHECK(apus_entries_to_nc_buf(log, &nc_lead));
    nc_fol = nc_lead;
    const uint64_t m = nc_lead.len ? splitmix() % nc_lead.len : 0;
    if (nc_lead.len) nc_fol.entries[m].term += 1;
    fwrite(&nc_fol.len, 1, 8, f);
    fwrite(nc_fol.entries, 24, nc_fol.len, f);
    fclose(f);
    CHECK(apus_find_remote_end(log, &nc_fol, &rend));

    printf("{\"n\": %u, \"commit_in\": %" PRIu64 ", \"new_commit\": %" PRIu64 ", \"committed\": %d, "
           "\"median\": %" PRIu64 ", \"publish\": %u, \"ssn\": %" PRIu64 ", \"remote_commit\": [%" PRIu64
           ", %" PRIu64 ", %" PRIu64 "], \"new_head\": %" PRIu64 ", \"append_head\": %d"
           ", \"won\": %d, \"vc\": [%u, %u], \"vote_commit\": %" PRIu64 ", \"voters\": %u, \"nc_len\": %" PRIu64
           ", \"nc_last\": [%" PRIu64 ", %" PRIu64 "], \"remote_end\": %" PRIu64 "}\n",
           n, commit0, new_commit, committed, median, post, ssn, rcommit[0], rcommit[1], rcommit[2], new_head,
           append_head, won, vc[0], vc[1], vcommit, voters, nc_lead.len,
           nc_lead.len ? nc_lead.entries[nc_lead.len - 1].idx : 0,
           nc_lead.len ? nc_lead.entries[nc_lead.len - 1].offset : 0, rend);
    CHECK(apus_log_free(log));
    return 0;
}
