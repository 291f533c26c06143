/*
 * ORACLE — TEST INFRASTRUCTURE ONLY.  Linked into oracle/_ref/libapusref.so
 * by oracle/Makefile, in this container only (it needs /root/reference).
 *
 * The proxy's stable-storage records on the REFERENCE's own
 *   /root/reference/src/include/proxy/proxy.h
 * (proxy_msg_header, proxy_send_msg, PROXY_SEND_MSG_SIZE,
 * PROXY_CONNECT_MSG_SIZE, PROXY_CLOSE_MSG_SIZE, CONNECT / SEND / CLOSE): the
 * bodies of stablestorage_save_request and stablestorage_load_records
 * (src/proxy/proxy.c:269-291, 306-339) restated on those types and macros.
 * The Berkeley DB underneath (store_record / dump_records,
 * src/db/db-interface.c:65-129: RECNO with DB_APPEND, dumped in record order)
 * is not in this image; its effect -- each stored record appended to the
 * snapshot -- is the sink below.  Lines marked BUILD-ONLY are the build's
 * documented stops where the reference reads past its buffers or spins
 * (include/apus_gpu.h); tests/test_transcription.py strips them before it
 * compares these bodies with the reference's token streams.
 *
 * This translation unit is separate from ref_compose.c: proxy.h's
 * common-header.h and dare_log.h's debug.h cannot share one unit.
 */
#include <stddef.h>
#include <stdint.h>
#include <string.h>

#include "proxy/proxy.h"   /* -I /root/reference/src/include */

/* the snapshot a store walk appends to (store_record's DB_APPEND, in order) */
typedef struct ref_rec_sink {
    uint8_t *buf;
    uint64_t cap;
    uint64_t len;
    uint32_t n;
    uint64_t avail;        /* bytes readable at the record's start (the log's end) */
    int stop;              /* BUILD-ONLY: a record past the log or the snapshot */
} ref_rec_sink;

static void sink_record(ref_rec_sink *s, size_t size, void *data)
{
    if (size > s->avail || s->len + size > s->cap) { s->stop = 1; return; }   /* BUILD-ONLY */
    memcpy(s->buf + s->len, data, size);
    s->len += size;
    s->n++;
}

/* stablestorage_save_request (proxy.c:269-291): the proxy_store_cmd callback
 * persist_new_entries hands &entry->clt_id (dare_server.c:1802) */
void ref_save_request(void *data, void *arg)
{
    /* TRANSCRIPTION save_request (proxy.c:271-290) */
    ref_rec_sink *sink = arg;
    proxy_msg_header *header = (proxy_msg_header *)data;
    switch (header->action) {
        case CONNECT:
        {
            sink_record(sink, PROXY_CONNECT_MSG_SIZE, data);
            break;
        }
        case SEND:
        {
            proxy_send_msg *send_msg = (proxy_send_msg *)data;
            if (sink->avail < sizeof(proxy_send_msg)) { sink->stop = 1; break; }   /* BUILD-ONLY */
            sink_record(sink, PROXY_SEND_MSG_SIZE(send_msg), data);
            break;
        }
        case CLOSE:
        {
            sink_record(sink, PROXY_CLOSE_MSG_SIZE, data);
            break;
        }
    }
    /* END TRANSCRIPTION save_request */
}

/* one snapshot's replay plan entry (apus_record_ref_t: offset u32, data_len
 * u32, connection_id u16, action u8, 5 pad) -- what do_action_send /
 * do_action_connect / do_action_close receive (proxy.c:317-333) */
typedef struct ref_plan {
    uint32_t offset, data_len;
    uint16_t connection_id;
    uint8_t action, pad[5];
} ref_plan;

/* the replay: the records a new server stores again (its store_record) and
 * the do_action_* calls, kept as plan entries */
typedef struct ref_replay {
    ref_plan *plan;
    uint32_t max_plan, n, at;
    uint32_t counts[3];
} ref_replay;

static void replay_store(ref_replay *r, size_t size, void *record) { (void)r; (void)size; (void)record; }
static void plan_entry(ref_replay *r, uint16_t conn, uint8_t action, uint32_t data_len)
{
    if (r->plan && r->n < r->max_plan) {
        ref_plan *p = &r->plan[r->n];
        memset(p, 0, sizeof *p);
        p->offset = r->at;
        p->data_len = data_len;
        p->connection_id = conn;
        p->action = action;
    }
    r->n++;
    r->counts[action - CONNECT]++;
}
static void plan_send(uint16_t conn, uint16_t len, uint8_t *cmd, void *arg)
{
    (void)cmd;
    plan_entry((ref_replay *)arg, conn, SEND, len);
}
static void plan_connect(uint16_t conn, void *arg) { plan_entry((ref_replay *)arg, conn, CONNECT, 0); }
static void plan_close(uint16_t conn, void *arg) { plan_entry((ref_replay *)arg, conn, CLOSE, 0); }

/* stablestorage_load_records (proxy.c:306-339) over one snapshot: the
 * do_action_* calls are recorded as plan entries (at most max_plan), the
 * per-action counts kept; returns the build-defined status (0 the whole
 * snapshot replayed, 1 an unknown action -- the reference's loop never
 * advances, 2 a record past `size` -- the reference reads past the buffer)
 * with *stop the bytes replayed */
int ref_records_load_one(const uint8_t *buf_in, uint32_t size, ref_plan *plan, uint32_t max_plan, uint32_t *n_out,
                         uint32_t counts[3], uint32_t *stop)
{
    ref_replay rp;
    memset(&rp, 0, sizeof rp);
    rp.plan = plan;
    rp.max_plan = max_plan;
    void *arg = &rp;
    void *buf = (void *)buf_in;
    int status = 0;
    /* TRANSCRIPTION load_records (proxy.c:308-337) */
    ref_replay *rec = arg;
    proxy_msg_header *header;
    uint32_t len = 0;
    while (len < size) {
        if (size - len < sizeof(proxy_msg_header)) { status = 2; break; }              /* BUILD-ONLY */
        header = (proxy_msg_header *)((char *)buf + len);
        rp.at = len;                                                                    /* BUILD-ONLY */
        if (header->action != SEND && header->action != CONNECT && header->action != CLOSE) { status = 1; break; }   /* BUILD-ONLY: the reference spins */
        if (header->action == SEND && size - len < offsetof(proxy_send_msg, data) + 2) { status = 2; break; }      /* BUILD-ONLY */
        if (header->action == SEND && PROXY_SEND_MSG_SIZE(((proxy_send_msg *)header)) > size - len) { status = 2; break; }   /* BUILD-ONLY */
        switch (header->action) {
            case SEND:
            {
                proxy_send_msg *send_msg = (proxy_send_msg *)header;
                len += PROXY_SEND_MSG_SIZE(send_msg);
                replay_store(rec, PROXY_SEND_MSG_SIZE(send_msg), header);
                plan_send(header->connection_id, send_msg->data.cmd.len, send_msg->data.cmd.cmd, arg);
                break;
            }
            case CONNECT:
            {
                len += PROXY_CONNECT_MSG_SIZE;
                replay_store(rec, PROXY_CONNECT_MSG_SIZE, header);
                plan_connect(header->connection_id, arg);
                break;
            }
            case CLOSE:
            {
                len += PROXY_CLOSE_MSG_SIZE;
                replay_store(rec, PROXY_CLOSE_MSG_SIZE, header);
                plan_close(header->connection_id, arg);
                break;
            }
        }
    }
    /* END TRANSCRIPTION load_records */
    *n_out = rp.n;
    counts[0] = rp.counts[0];
    counts[1] = rp.counts[1];
    counts[2] = rp.counts[2];
    *stop = len;
    return status;
}

/* the sink the store walk in ref_compose.c fills (opaque there) */
size_t ref_rec_sink_size(void) { return sizeof(ref_rec_sink); }
void ref_rec_sink_init(void *s, uint8_t *buf, uint64_t cap, uint64_t len)
{
    ref_rec_sink *k = (ref_rec_sink *)s;
    memset(k, 0, sizeof *k);
    k->buf = buf;
    k->cap = cap;
    k->len = len;
}
void ref_rec_sink_avail(void *s, uint64_t avail) { ((ref_rec_sink *)s)->avail = avail; }
int ref_rec_sink_stopped(const void *s) { return ((const ref_rec_sink *)s)->stop; }
uint64_t ref_rec_sink_len(const void *s) { return ((const ref_rec_sink *)s)->len; }
uint32_t ref_rec_sink_n(const void *s) { return ((const ref_rec_sink *)s)->n; }
