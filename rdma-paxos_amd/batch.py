"""Group-major batch containers: numpy on the host, torch on the device.

Layout (identical on both sides, see include/apus_gpu.h apus_batch_t):
  ring            uint8   [G * ring_stride]   each group's dare_log_t.entries[] image
  state           64 B    [G]                 head, apply, commit, end, tail, len, cid
  self_idx        uint8   [G]                 config.idx
  remote_end      uint64  [G, R]              ctrl_data->log_offsets[i].end
  remote_commit   uint64  [G, R]              ctrl_data->log_offsets[i].commit
  lr_step         uint8   [G, R]              servers[i].next_lr_step
  fail_count      uint8   [G, R]              servers[i].fail_count
  vote_ack        uint64  [G, R]              ctrl_data->vote_ack[i]
  apply_offsets   uint64  [G, R]              ctrl_data->apply_offsets[i]
  vote_req        40 B    [G, R]              ctrl_data->vote_req[i]
  hb              uint64  [G, R]              ctrl_data->hb[i]
  sid             uint64  [G]                 ctrl_data->sid
  last_idx_term   uint64  [G, 2]              local last (idx, term)
  prev_head       uint8   [G]                 prev_log_entry_head
  abs_base        uint64  [G]                 absolute position of ring offset 0
  rc_connected    uint16  [G]                 bit i = servers[i].ep->rc_connected (opt-in)
  vote_sit        uint64  [G][R][3]           vote_req[i]'s (sid, index, term) packed (opt-in; fill_vote_sit)
"""
import ctypes as C

import numpy as np

from . import abi

CID_DT = np.dtype([("epoch", "<u8"), ("size0", "u1"), ("size1", "u1"), ("state", "u1"),
                   ("pad", "u1"), ("bitmask", "<u4")])
STATE_DT = np.dtype([("head", "<u8"), ("apply", "<u8"), ("commit", "<u8"), ("end", "<u8"),
                     ("tail", "<u8"), ("len", "<u8"), ("cid", CID_DT)])
VOTE_REQ_DT = np.dtype([("sid", "<u8"), ("index", "<u8"), ("term", "<u8"), ("cid", CID_DT)])
DET_DT = np.dtype([("idx", "<u8"), ("term", "<u8"), ("offset", "<u8")])
APPEND_DT = np.dtype([("req_id", "<u8"), ("data_off", "<u8"), ("clt_id", "<u2"), ("type", "u1"),
                      ("pad", "u1", (5,))])
assert STATE_DT.itemsize == 64 and VOTE_REQ_DT.itemsize == 40 and DET_DT.itemsize == 24
assert APPEND_DT.itemsize == 24

# (field, numpy dtype, elements per group as a function of R)
FIELDS = [
    ("state", STATE_DT, lambda R: 1),
    ("self_idx", np.uint8, lambda R: 1),
    ("remote_end", np.uint64, lambda R: R),
    ("remote_commit", np.uint64, lambda R: R),
    ("lr_step", np.uint8, lambda R: R),
    ("fail_count", np.uint8, lambda R: R),
    ("vote_ack", np.uint64, lambda R: R),
    ("apply_offsets", np.uint64, lambda R: R),
    ("vote_req", VOTE_REQ_DT, lambda R: R),
    ("hb", np.uint64, lambda R: R),
    ("sid", np.uint64, lambda R: 1),
    ("last_idx_term", np.uint64, lambda R: 2),
    ("prev_head", np.uint8, lambda R: 1),
    ("abs_base", np.uint64, lambda R: 1),
    ("rc_connected", np.uint16, lambda R: 1),
    ("vote_sit", np.uint64, lambda R: 3 * R),
]
# rc_connected and vote_sit are opt-in (a NULL rc_connected means every
# server is connected; a NULL vote_sit makes the ranking read vote_req)
OPT_IN = ("rc_connected", "vote_sit")
ALL_FIELDS = [f[0] for f in FIELDS if f[0] not in OPT_IN]


def ring_stride_for(ring_len):
    """stride >= len + 16 (the window loads may read up to 15 bytes past len)"""
    return (ring_len + 16 + 15) // 16 * 16


def gen_cfg(seed=1, gid_base=0, n_entries=64, n_history=16, len_min=64, len_max=64,
            ring_len=16384, p_full_ack=0.9, straggler=False, type_mix=False, cid_mix=False,
            garbage_reply=0.0, self_random=False, p_vote_ack=0.6, hist_len_max=0):
    return abi.GenCfg(seed=seed, gid_base=gid_base, n_entries=n_entries, n_history=n_history,
                      len_min=len_min, len_max=len_max, ring_len=ring_len,
                      p_full_ack=int(round(p_full_ack * 65536)), straggler=int(straggler),
                      type_mix=int(type_mix), cid_mix=int(cid_mix),
                      garbage_reply=int(round(garbage_reply * 65536)),
                      self_random=int(self_random),
                      p_vote_ack=int(round(p_vote_ack * 65536)), fill_garbage=1, hist_len_max=hist_len_max)


class HostBatch:
    """numpy-backed batch (oracle side)."""

    def __init__(self, n_groups, n_replicas, ring_stride, fields=ALL_FIELDS):
        self.G, self.R, self.stride = int(n_groups), int(n_replicas), int(ring_stride)
        self.ring = np.zeros(self.G * self.stride, dtype=np.uint8)
        self.arrays = {}
        for name, dt, per in FIELDS:
            if name in fields:
                self.arrays[name] = np.zeros(self.G * per(self.R), dtype=dt)

    def __getattr__(self, k):
        a = self.__dict__.get("arrays", {})
        if k in a:
            return a[k]
        raise AttributeError(k)

    def struct(self):
        b = abi.Batch(n_groups=self.G, n_replicas=self.R, flags=0, ring_stride=self.stride)
        b.ring = self.ring.ctypes.data
        for name, arr in self.arrays.items():
            setattr(b, name, arr.ctypes.data)
        return b

    def group_ring(self, g):
        return self.ring[g * self.stride:(g + 1) * self.stride]

    def add(self, name):
        """allocate an opt-in field (e.g. rc_connected), zeroed"""
        dt, per = {f[0]: (f[1], f[2]) for f in FIELDS}[name]
        self.arrays[name] = np.zeros(self.G * per(self.R), dtype=dt)
        return self.arrays[name]

    def fill_vote_sit(self):
        """vote_sit from vote_req: each record's (sid, index, term), packed"""
        if "vote_sit" not in self.arrays:
            self.add("vote_sit")
        vr = self.arrays["vote_req"]
        s = self.arrays["vote_sit"].reshape(-1, 3)
        s[:, 0], s[:, 1], s[:, 2] = vr["sid"], vr["index"], vr["term"]
        return self.arrays["vote_sit"]


class DeviceBatch:
    """torch-backed batch resident in HBM (product side)."""

    def __init__(self, n_groups, n_replicas, ring_stride, device="cuda", fields=ALL_FIELDS):
        import torch
        self.torch = torch
        self.G, self.R, self.stride = int(n_groups), int(n_replicas), int(ring_stride)
        self.device = device
        self.ring = torch.empty(self.G * self.stride, dtype=torch.uint8, device=device)
        self.arrays = {}
        for name, dt, per in FIELDS:
            if name in fields:
                nbytes = self.G * per(self.R) * np.dtype(dt).itemsize
                self.arrays[name] = torch.zeros(nbytes, dtype=torch.uint8, device=device)

    def struct(self):
        b = abi.Batch(n_groups=self.G, n_replicas=self.R, flags=0, ring_stride=self.stride)
        b.ring = self.ring.data_ptr()
        for name, t in self.arrays.items():
            setattr(b, name, t.data_ptr())
        return b

    def add(self, name):
        """allocate an opt-in field (e.g. rc_connected), zeroed"""
        dt, per = {f[0]: (f[1], f[2]) for f in FIELDS}[name]
        self.arrays[name] = self.torch.zeros(self.G * per(self.R) * np.dtype(dt).itemsize, dtype=self.torch.uint8,
                                             device=self.device)
        return self.arrays[name]

    def fill_vote_sit(self):
        """vote_sit from vote_req on the device: each 40-B record's first 24 B
        (sid, index, term), packed (outside any timed region)"""
        if "vote_sit" not in self.arrays:
            self.add("vote_sit")
        vr = self.arrays["vote_req"].view(self.torch.int64).view(-1, 5)
        self.arrays["vote_sit"].view(self.torch.int64).view(-1, 3).copy_(vr[:, :3])
        return self.arrays["vote_sit"]

    def upload(self, host):
        assert (host.G, host.R, host.stride) == (self.G, self.R, self.stride)
        self.ring.copy_(self.torch.from_numpy(host.ring))
        for name, t in self.arrays.items():
            if name in host.arrays:
                t.copy_(self.torch.from_numpy(host.arrays[name].view(np.uint8)))

    def download(self, name):
        """numpy copy of a field with its host dtype"""
        if name == "ring":
            return self.ring.cpu().numpy()
        dt = dict((f[0], f[1]) for f in FIELDS)[name]
        return self.arrays[name].cpu().numpy().view(dt)


def log_image_stride(ring_len):
    """bytes per dare_log_t image: the 319,656-B header, the ring, the 16-B
    tail pad the 16-B window loads may touch, rounded to 256 B"""
    return (abi.LOG_HDR_BYTES + ring_len + 16 + 255) // 256 * 256


class LogImageBatch:
    """G device-resident dare_log_t images (dare_log.h:77-103) -- the layout
    the reference registers for RDMA -- plus the per-replica columns of a
    DeviceBatch (APUS_BATCH_LOG_IMAGE).  Images start at 8 mod 16 so each
    entries[] is 16-B aligned.  header(g) / entries(g) are byte views of
    group g's header and ring."""

    HDR_FIELDS = ("head", "apply", "commit", "end", "tail", "old_end", "old_commit", "len")

    def __init__(self, n_groups, n_replicas, ring_len, device="cuda", fields=ALL_FIELDS):
        import torch
        self.torch = torch
        self.G, self.R, self.L = int(n_groups), int(n_replicas), int(ring_len)
        self.stride = log_image_stride(self.L)
        self.buf = torch.zeros(self.G * self.stride + 256, dtype=torch.uint8, device=device)
        self.off = (-(self.buf.data_ptr() + abi.LOG_HDR_BYTES)) % 16
        self.images = self.buf[self.off:self.off + self.G * self.stride].view(self.G, self.stride)
        self.cid = torch.zeros(self.G * 16, dtype=torch.uint8, device=device)
        self.cols = DeviceBatch(self.G, self.R, 16, device=device,
                                fields=[f for f in fields if f not in ("state",)])
        self.cols.ring = self.cols.ring[:0]

    def header(self, g=None):
        h = self.images[:, :64].contiguous().view(self.torch.int64).view(self.G, 8)
        return h if g is None else h[g]

    def fill_from(self, host):
        """copy a HostBatch (state rows + rings) into the images: header
        offsets from the state row (old_end = end, old_commit = commit),
        entries[] = the ring, config.cid into cid"""
        t = self.torch
        assert (host.G, host.R) == (self.G, self.R)
        st = host.state
        hdr = np.zeros((self.G, 8), np.uint64)
        for k, name in enumerate(self.HDR_FIELDS):
            src = {"old_end": "end", "old_commit": "commit"}.get(name, name)
            hdr[:, k] = st[src]
        dev = self.images.device
        self.images[:, :64] = t.from_numpy(hdr.view(np.uint8).reshape(self.G, 64)).to(dev)
        rings = t.from_numpy(host.ring.reshape(self.G, host.stride)[:, :self.L].copy()).to(dev)
        self.images[:, abi.LOG_HDR_BYTES:abi.LOG_HDR_BYTES + self.L] = rings
        self.cid.copy_(t.from_numpy(np.ascontiguousarray(st["cid"]).view(np.uint8).reshape(-1)).to(dev))
        for name, tt in self.cols.arrays.items():
            if name in host.arrays:
                tt.copy_(t.from_numpy(host.arrays[name].view(np.uint8)))

    def entries_ptr(self):
        return self.images.data_ptr() + abi.LOG_HDR_BYTES

    def download(self, name):
        """numpy copy: "state" as state rows rebuilt from the image headers
        (head, apply, commit, end, tail, len@56) and the cid array; "ring" as
        [G, L] entries[] bytes; any other name from the replica columns"""
        if name == "state":
            h = self.images[:, :64].contiguous().cpu().numpy().view(np.uint64).reshape(self.G, 8)
            st = np.zeros(self.G, STATE_DT)
            for k, f in enumerate(("head", "apply", "commit", "end", "tail")):
                st[f] = h[:, k]
            st["len"] = h[:, 7]
            st["cid"] = self.cid.cpu().numpy().view(CID_DT)
            return st
        if name == "ring":
            return self.images[:, abi.LOG_HDR_BYTES:abi.LOG_HDR_BYTES + self.L].contiguous().cpu().numpy()
        return self.cols.download(name)

    def struct(self):
        b = self.cols.struct()
        b.n_groups, b.n_replicas = self.G, self.R
        b.flags = abi.BATCH_LOG_IMAGE
        b.ring_stride = self.stride
        b.ring = self.entries_ptr()
        b.state = None
        b.cid = self.cid.data_ptr()
        return b


def device_out(torch, G, spec, device="cuda"):
    """allocate output tensors: spec = {name: (torch dtype, per-group count)}"""
    return {k: torch.zeros(G * n, dtype=dt, device=device) for k, (dt, n) in spec.items()}


def ptr(t):
    return None if t is None else t.data_ptr()


def make_messages(G, M, seed=1, len_min=64, len_max=64, type_mix=False, align=1, scatter=False):
    """Synthetic client messages for apus_append_batch: G queues of M
    messages (APPEND_DT records) plus the payload arena their data_off
    index -- an sm_cmd_t {u16 len; cmd[len]} per CSM-class message, a 16-B
    dare_cid_t per CONFIG, an 8-B head per HEAD.  type_mix draws NOOP /
    CONFIG / HEAD / CONNECT(4) / SEND(5) / CLOSE(6), else all SEND.  Each
    record starts at a multiple of `align` bytes of the arena; the records
    lie in queue order, or in a random order with `scatter`."""
    rng = np.random.default_rng(seed)
    n = G * M
    if type_mix:
        types = rng.choice(np.array([0, 2, 3, 4, 5, 6], np.uint8), size=n,
                           p=[0.06, 0.06, 0.06, 0.06, 0.70, 0.06])
    else:
        types = np.full(n, 5, np.uint8)
    csm = ~np.isin(types, (0, 2, 3))
    clen = rng.integers(len_min, len_max + 1, size=n).astype(np.int64)
    need = np.where(csm, 2 + clen, np.where(types == 2, 16, np.where(types == 3, 8, 0)))
    need = (need + (align - 1)) // align * align
    order = rng.permutation(n) if scatter else np.arange(n)
    off = np.zeros(n, np.int64)
    if n > 1:
        off[order[1:]] = np.cumsum(need[order][:-1])
    total = int(need.sum())
    payload = rng.integers(0, 256, size=max(total, 1), dtype=np.uint8)
    o = off[csm]
    payload[o] = (clen[csm] & 0xFF).astype(np.uint8)
    payload[o + 1] = (clen[csm] >> 8).astype(np.uint8)
    ent = np.zeros(n, APPEND_DT)
    ent["req_id"] = rng.integers(0, 1 << 62, size=n, dtype=np.uint64)
    ent["data_off"] = off.astype(np.uint64)
    ent["clt_id"] = rng.integers(0, 1 << 16, size=n, dtype=np.uint16)
    ent["type"] = types
    return ent, payload
