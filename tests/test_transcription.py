"""Transcription drift (VERDICT r3 #6b): the loop bodies oracle/_ref restates
on top of the reference's compiled primitives (oracle/ref_compose.c,
oracle/ref_records.c) against the reference's own source text.

Container only: the reference tree is read as text (skipped where it is
absent, e.g. on the GPU box).  Each region pairs a cited line range of the
reference with a marked region of ours (/* TRANSCRIPTION name */ ...
/* END TRANSCRIPTION name */).  Both are reduced to the same skeleton and
must be equal token for token:
  * comments, disabled preprocessor branches (#if 0 / the #else of #if 1) and
    other preprocessor lines go; the reference's logging / timer statements
    (info, text, TIMER_*, ...) go; our BUILD-ONLY lines (the build's
    documented stops where the reference spins or reads past its buffers) go;
  * member-access chains become one path token (index expressions replaced
    by [] and emitted after it), renamed through the region's committed map
    (the reference's SRV_DATA->ctrl_data->log_offsets[].end and our rend[]
    both become REND[]); a path in neither map must be spelled the same on
    both sides;
  * types, declarations' type words, braces, parentheses, commas, semicolons,
    unary & and * are dropped; keywords, operators, literals, constants and
    the calls to the reference's primitives stay, in order.
So any change to a comparison, an operator, a literal, the order of a
primitive's arguments or the control flow, on either side, fails here.
"""
import os
import re

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
REF = "/root/reference"

DROP_WORDS = {"int", "uint8_t", "uint16_t", "uint32_t", "uint64_t", "const", "static", "char", "void", "unsigned",
              "struct", "dare_log_entry_t", "proxy_msg_header", "proxy_send_msg", "size_t", "register"}
DROP_CALLS = {"info", "text", "debug", "info_wtime", "TIMER_INIT", "TIMER_START", "TIMER_STOP", "TIMER_INFO", "PRINT_SID_",
              "HRT_GET_TIMESTAMP", "HRT_GET_ELAPSED_TICKS", "PRINT_CONF_TRANSIT",
              "INFO_PRINT_LOG"}
DROP_TOKENS = {","}
# '*' and '&' are dropped where they are unary (dereference, address-of: the
# transcriptions hold values where the reference holds pointers) and kept
# where they are binary (multiplication, bitwise and)
UNARY_CTX = {"(", "[", "{", "}", ";", ",", "=", "==", "!=", "<", ">", "<=", ">=", "&&", "||", "!", "return", "?",
             ":", "+", "-", "+=", "-=", "*", "/", "%", "&", "|", "^", "~", "<<", ">>"}
TOKEN = re.compile(r"[A-Za-z_]\w*|0[xX][0-9a-fA-F]+[uUlL]*|\d+[uUlL]*|->|\+\+|--|<=|>=|==|!=|&&|\|\||\+=|-=|<<|>>|"
                   r"[-+*/%<>=!&|^~?:.,;(){}\[\]]")


def strip_c(text):
    """comments, then preprocessor: the bodies of #if 0 and the #else of
    #if 1 go, every directive line goes (other conditionals keep their first
    branch)"""
    text = re.sub(r"/\*.*?\*/", " ", text, flags=re.S)
    text = re.sub(r"//[^\n]*", "", text)
    # string literals (format strings hold ';'): one token, before the
    # logging calls that carry them are dropped
    text = re.sub(r'"(?:\\.|[^"\\\n])*"', " STRLIT ", text)
    out, stack = [], []
    for line in text.split("\n"):
        s = line.strip().replace(" ", "")
        if s.startswith("#if"):
            stack.append(s != "#if0")
        elif s.startswith("#else"):
            if stack:
                stack[-1] = not stack[-1]
        elif s.startswith("#endif"):
            if stack:
                stack.pop()
        elif s.startswith("#"):
            continue
        elif all(stack):
            out.append(line)
    return "\n".join(out)


def tokens(text):
    return TOKEN.findall(text)


def drop_statements(toks):
    """the reference's logging / timer calls, each up to its ';'"""
    out, i = [], 0
    while i < len(toks):
        if toks[i] in DROP_CALLS:
            while i < len(toks) and toks[i] != ";":
                i += 1
            i += 1
            continue
        out.append(toks[i])
        i += 1
    return out


def unary_drop(toks):
    """unary '*' / '&' out (after an operator, a punctuator, a type word or
    at the start); binary ones stay"""
    out = []
    for k, t in enumerate(toks):
        if t in ("*", "&"):
            prev = toks[k - 1] if k else None
            if prev is None or prev in UNARY_CTX or prev in DROP_WORDS:
                continue
        out.append(t)
    return out


def skeleton(toks, rename):
    """paths (a->b.c[i].d) renamed, index expressions after them; dropped
    tokens out (commas, unary '*' / '&', type words); parentheses, braces and
    semicolons stay, so precedence and statement structure are compared"""
    toks = unary_drop(toks)
    out = []

    def expr(i, stop):
        while i < len(toks) and toks[i] != stop:
            i = primary(i)
        return i

    def primary(i):
        t = toks[i]
        if not re.match(r"[A-Za-z_]", t) or t in DROP_WORDS:
            if t not in DROP_TOKENS and t not in DROP_WORDS:
                out.append(t)
            return i + 1
        path, idx = t, []
        i += 1
        while i < len(toks):
            if toks[i] in ("->", ".") and i + 1 < len(toks):
                path += "." + toks[i + 1]
                i += 2
            elif toks[i] == "[":
                j, depth = i + 1, 1
                while depth:
                    depth += {"[": 1, "]": -1}.get(toks[j], 0)
                    j += 1
                idx.append(toks[i + 1:j - 1])
                path += "[]"
                i = j
            else:
                break
        out.append(rename.get(path, path))
        for sub in idx:
            sk = skeleton(sub, rename)
            out.extend(sk)
        return i

    i = 0
    while i < len(toks):
        i = primary(i)
    return out


def ref_region(path, a, b):
    with open(os.path.join(REF, path)) as f:
        lines = f.read().split("\n")
    return drop_statements(tokens(strip_c("\n".join(lines[a - 1:b]))))


def our_region(path, name):
    with open(os.path.join(ROOT, path)) as f:
        text = f.read()
    m = re.search(r"/\* TRANSCRIPTION %s\b[^*]*\*/(.*?)/\* END TRANSCRIPTION %s \*/" % (name, name), text, re.S)
    assert m, f"{path}: no region {name}"
    body = "\n".join(l for l in m.group(1).split("\n") if "BUILD-ONLY" not in l)
    return drop_statements(tokens(strip_c(body)))


# name: (reference file, first line, last line, our file, reference renames, our renames)
REGIONS = {
    # APUS reply-count commit walk, update_remote_logs (a3)
    "walk": ("src/dare/dare_ibv_rc.c", 1725, 1758, "oracle/ref_compose.c",
             {"min_offset": "MO", "SRV_DATA.log": "LOG", "SRV_DATA.log.commit": "COMMIT", "SRV_DATA.config.idx": "SELF",
              "dare_log_entry_t": "", "entry.reply[]": "REPLY[]", "SRV_DATA.config.cid_offset": "CIDOFF"},
             {"mo": "MO", "log": "LOG", "log.commit": "COMMIT", "cfg.idx": "SELF", "entry.reply[]": "REPLY[]",
              "cfg.cid_offset": "CIDOFF"}),
    # DARE median-offset quorum (a4)
    "median": ("src/dare/dare_ibv_rc.c", 1652, 1723, "oracle/ref_compose.c",
               {"SRV_DATA.log.commit": "COMMIT", "SRV_DATA.log.end": "END", "SRV_DATA.log": "LOG",
                "SRV_DATA.config.cid.size[]": "CIDSIZE[]", "SRV_DATA.config.idx": "SELF",
                "SRV_DATA.config.cid": "CID", "SRV_DATA.config.cid.state": "CIDSTATE",
                "SRV_DATA.config.servers[].fail_count": "FAIL[]", "SRV_DATA.config.servers[].next_lr_step": "STEP[]",
                "SRV_DATA.ctrl_data.log_offsets[].end": "REND[]", "larger_offset_count": "CNT",
                "PERMANENT_FAILURE": "2", "LR_UPDATE_LOG": "5"},
               {"log.commit": "COMMIT", "log.end": "END", "log": "LOG", "cfg.cid.size[]": "CIDSIZE[]",
                "cfg.idx": "SELF", "cfg.cid": "CID", "cfg.cid.state": "CIDSTATE", "fail[]": "FAIL[]",
                "step[]": "STEP[]", "rend[]": "REND[]", "cnt": "CNT"}),
    # poll_vote_count (a5)
    "vote": ("src/dare/dare_server.c", 1332, 1373, "oracle/ref_compose.c",
             {"data.config": "CFG", "data.config.idx": "SELF", "data.ctrl_data.vote_ack[]": "ACK[]",
              "data.log.len": "LEN", "data.config.cid.size[]": "CIDSIZE[]", "data.log": "LOG",
              "data.log.commit": "COMMIT", "data.config.cid.state": "CIDSTATE", "remote_commit": "RC",
              "vote_count[]": "VC[]", "data.ctrl_data.log_offsets[].commit": "VOTED[]",
              "data.config.servers[].next_lr_step": "VSTEP[]", "LR_GET_NCE_LEN": "2"},
             {"cfg": "CFG", "cfg.idx": "SELF", "vote_ack[]": "ACK[]", "log.len": "LEN", "cfg.cid.size[]": "CIDSIZE[]",
              "log": "LOG", "log.commit": "COMMIT", "cfg.cid.state": "CIDSTATE", "rc": "RC", "vc[]": "VC[]",
              "voted[]": "VOTED[]", "vstep[]": "VSTEP[]"}),
    # log_pruning's minimum (a7)
    "prune": ("src/dare/dare_server.c", 2026, 2050, "oracle/ref_compose.c",
              {"data.config": "CFG", "data.log.apply": "APPLY", "data.config.cid": "CID",
               "data.ctrl_data.apply_offsets[]": "AP[]", "data.log": "LOG", "data.log.head": "HEAD",
               "min_offset": "MIN", "prev_log_entry_head": "PREV"},
              {"cfg": "CFG", "log.apply": "APPLY", "cfg.cid": "CID", "apply_offsets[]": "AP[]", "log": "LOG",
               "log.head": "HEAD", "min_offset": "MIN", "prev_head": "PREV"}),
    # persist_new_entries' walk feeding the stable-storage records (8f.3)
    "persist": ("src/dare/dare_server.c", 1796, 1802, "oracle/ref_compose.c",
                {"data.log": "LOG", "data.log.end": "END", "data.log.old_end": "OE",
                 "data.sm.proxy_store_cmd": "STORE", "entry.clt_id": "CLT", "data.sm.up_para": "SINK"},
                {"log": "LOG", "log.end": "END", "log.old_end": "OE", "ref_save_request": "STORE",
                 "entry.clt_id": "CLT", "sink": "SINK"}),
    # poll_vote_requests (a6): the leader / heartbeat tests and the best SID
    "rank_best": ("src/dare/dare_server.c", 1535, 1579, "oracle/ref_compose.c",
                  {"data.ctrl_data.sid": "SID", "data.ctrl_data.hb[]": "HB[]", "data.ctrl_data.vote_req[]": "REQ[]",
                   "data.config.idx": "SELF"},
                  {"ctrl.sid": "SID", "ctrl.hb[]": "HB[]", "ctrl.vote_req[]": "REQ[]", "cfg.idx": "SELF"}),
    # ... the candidate's local (idx, term)
    "rank_local": ("src/dare/dare_server.c", 1598, 1620, "oracle/ref_compose.c",
                   {"data.log.nc_buf[]": "NCB[]", "data.config.idx": "SELF", "data.log": "LOG",
                    "data.log.len": "LEN"},
                   {"nc_store[]": "NCB[]", "self": "SELF", "log": "LOG", "log.len": "LEN"}),
    # ... and the up-to-date test over every request
    "rank_uptodate": ("src/dare/dare_server.c", 1626, 1668, "oracle/ref_compose.c",
                      {"data.ctrl_data.sid": "SID", "data.ctrl_data.vote_req[]": "REQ[]", "data.config.idx": "SELF"},
                      {"ctrl.sid": "SID", "ctrl.vote_req[]": "REQ[]", "cfg.idx": "SELF"}),
    # poll_config_entries and update_cid (8f.2)
    "config_scan": ("src/dare/dare_server.c", 2136, 2186, "oracle/ref_compose.c", {}, {}),
    "update_cid": ("src/dare/dare_server.c", 2195, 2226, "oracle/ref_compose.c", {}, {}),
    # apply_committed_entries (8f.2): the CONFIG re-append is recorded
    "apply": ("src/dare/dare_server.c", 1821, 1973, "oracle/ref_compose.c",
              {"log_append_entry": "APPEND"}, {"cfg_append": "APPEND"}),
    # log_adjustment (8f.2): post_send records the work request
    "log_adjust": ("src/dare/dare_ibv_rc.c", 1313, 1446, "oracle/ref_compose.c", {}, {}),
    # handle_lr_work_completion (8f.2)
    "lr_completion": ("src/dare/dare_ibv_rc.c", 3137, 3194, "oracle/ref_compose.c", {}, {}),
    # update_remote_logs' lazy remote-commit publish (the post of the write is recorded)
    "publish": ("src/dare/dare_ibv_rc.c", 1761, 1794, "oracle/ref_compose.c", {}, {}),
    # force_log_pruning (polling(), dare_server.c:1123)
    "force_prune": ("src/dare/dare_server.c", 2073, 2121, "oracle/ref_compose.c", {}, {}),
    # poll_vote_count whole: the tally, then the election-win transition
    # (SID L bit, config scan, apply, the blank entry, become_leader)
    "vote_count": ("src/dare/dare_server.c", 1332, 1510, "oracle/ref_compose.c", {}, {}),
    # stablestorage_save_request (8f.3)
    "save_request": ("src/proxy/proxy.c", 271, 290, "oracle/ref_records.c",
                     {"proxy": "SINK", "arg": "ARG", "store_record": "STORE", "proxy.db_ptr": "SINK",
                      "proxy_node": ""},
                     {"sink": "SINK", "arg": "ARG", "sink_record": "STORE", "ref_rec_sink": ""}),
    # stablestorage_load_records (8f.3): the new server's store_record and
    # do_action_* calls are the replay's store and plan entries
    "load_records": ("src/proxy/proxy.c", 308, 337, "oracle/ref_records.c",
                     {"proxy_node": "", "proxy": "DB", "arg": "ARG", "store_record": "STORE", "proxy.db_ptr": "DB",
                      "do_action_send": "PLAN_SEND", "do_action_connect": "PLAN_CONNECT",
                      "do_action_close": "PLAN_CLOSE"},
                     {"ref_replay": "", "rec": "DB", "arg": "ARG", "replay_store": "STORE", "plan_send": "PLAN_SEND",
                      "plan_connect": "PLAN_CONNECT", "plan_close": "PLAN_CLOSE"}),
}


@pytest.mark.skipif(not os.path.isdir(REF), reason="reference tree absent on this machine")
@pytest.mark.parametrize("name", list(REGIONS))
def test_transcription_matches_reference(name):
    rf, a, b, ours, rmap, omap = REGIONS[name]
    r = [t for t in skeleton(ref_region(rf, a, b), rmap) if t]
    o = [t for t in skeleton(our_region(ours, name), omap) if t]
    if r != o:
        import difflib
        d = "\n".join(difflib.unified_diff(r, o, "reference", "ours", lineterm="", n=4))
        pytest.fail(f"{name}: {rf}:{a}-{b} and {ours} differ:\n{d}")


def test_skeleton_catches_drift():
    """the reduction keeps what matters: a flipped comparison, a swapped
    argument, a changed literal, an operator, the parenthesisation (operator
    precedence) and the statement structure change the skeleton"""
    base = "while (log_is_offset_larger(log, a, b)) { if (x < size / 2 + 1) break; y = 0.75 * n; }"
    sk = skeleton(tokens(base), {})
    for mutant in ("while (log_is_offset_larger(log, b, a)) { if (x < size / 2 + 1) break; y = 0.75 * n; }",
                   "while (log_is_offset_larger(log, a, b)) { if (x <= size / 2 + 1) break; y = 0.75 * n; }",
                   "while (log_is_offset_larger(log, a, b)) { if (x < size / 2 + 2) break; y = 0.75 * n; }",
                   "while (log_is_offset_larger(log, a, b)) { if (x < size / 2 + 1) continue; y = 0.75 * n; }",
                   "while (log_is_offset_larger(log, a, b)) { if (x < size / (2 + 1)) break; y = 0.75 * n; }",
                   "while (log_is_offset_larger(log, a, b)) { if (x < size / 2 + 1) break; y = 0.75 + n; }",
                   "while (log_is_offset_larger(log, a, b)) { if (x < size / 2 + 1) break; } y = 0.75 * n;",
                   "while (log_is_offset_larger(log, a, b)) { if (x < size / 2 + 1) { break; y = 0.75 * n; } }"):
        assert skeleton(tokens(mutant), {}) != sk, mutant
    # what it ignores: layout, types, comments, commas, unary * and &
    same = "/* c */ while ( log_is_offset_larger ( log , a , b ) )\n{ if (x < size / 2 + 1) break;\n y = 0.75 * n; }"
    assert skeleton(tokens(strip_c(same)), {}) == sk
    assert skeleton(tokens("*p = &q->r; z = a * b & c;"), {}) == skeleton(tokens("p = q->r; z = a * b & c;"), {})
    assert skeleton(tokens("uint64_t *p = x;"), {}) == skeleton(tokens("uint64_t p = x;"), {})
