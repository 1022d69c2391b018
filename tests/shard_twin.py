"""CPU twin of shard.DeviceShardOps for the world-2 gloo tests of shard.ingest_sharded (no GPU
in this container): the product's host twins compute the gate (ce_shard_stats_host,
ce_shard_window_host -- the same math as the device kernels, tests/test_gpu_shard.py compares
them), and the oracle (oracle/ce_oracle.c, the reference restatement) opens, checks and folds
each file.  The committed state is a dense GCounter over the writer table, serialized as the
product's StateWrapper<GCounter> bytes (crdt-enc/src/lib.rs:739-743)."""
import msgpack
import numpy as np
import torch

import crdtenc
import shard

APP = bytes.fromhex("aadfd5a66e194b24a8024fa27c72f20c")


class TwinCore:
    """state_bytes / merge_state over a dict GCounter (the bytes exchange path)."""

    def __init__(self):
        self.state, self.nov = {}, {}

    def fold_bytes(self, ser):
        d = msgpack.unpackb(ser, raw=True, strict_map_key=False)
        for a, c in d[b"state"][b"inner"][b"dots"].items():
            self.state[a] = max(self.state.get(a, 0), c)
        for a, c in d[b"next_op_versions"][b"dots"].items():
            self.nov[a] = max(self.nov.get(a, 0), c)

    def state_bytes(self):
        return msgpack.packb({"next_op_versions": {"dots": dict(sorted(self.nov.items()))},
                              "state": {"inner": {"dots": dict(sorted(self.state.items()))}}},
                             use_bin_type=True)

    def merge_state(self, sw):
        self.fold_bytes(sw)
        return 0


class HostShardOps:
    """One rank: files[i] written by writers[fa[i]] at version fv[i] (its partition's share);
    registered = the actors with dense slots (in order)."""

    def __init__(self, core, key, writers, registered, files, fa, fv):
        self.core, self.key = core, key
        self.writers = list(writers)
        self.actors = b"".join(self.writers)
        self.reg = list(registered)
        self.files = list(files)
        self.fa = np.asarray(fa, np.uint32)
        self.fv = np.asarray(fv, np.uint64)
        self.pending = None

    def writer_versions(self):
        return np.array([self.core.nov.get(w, 0) for w in self.writers], np.uint64)

    def compute_stats(self, rank, world):
        st = crdtenc.shard_stats_host(self.writers, self.writer_versions(), self.fa, self.fv, rank, world)
        self.stats = torch.from_numpy(st.copy())
        return self.stats

    def window(self):
        self.hi, self.flags = crdtenc.shard_window_host(self.writer_versions(), self.stats.numpy())

    def set_window(self, hi, flags):
        self.hi, self.flags = np.asarray(hi, np.uint64), flags

    def metadata(self):
        return self.fa, self.fv

    def ingest(self):
        import oracle
        self.pending = None
        if self.flags & (shard.SHARD_BAD | shard.SHARD_E0_MISMATCH):
            return shard.ERR_SHARD
        e0 = self.writer_versions()
        batch = TwinCore()
        for i, f in enumerate(self.files):  # every file opens and decodes, applied or not
            oc = oracle.Core(oracle.STATE_GCOUNTER)
            rc, _ = oc.read_remote_ops(self.key, [APP], [f], [self.writers[self.fa[i]]], [0])
            if rc:
                return rc
            a = int(self.fa[i])
            if e0[a] <= self.fv[i] < self.hi[a]:
                d = msgpack.unpackb(oc.serialize(), raw=True, strict_map_key=False)
                for x, c in d[b"state"][b"inner"][b"dots"].items():
                    batch.state[x] = max(batch.state.get(x, 0), c)
        for a, w in enumerate(self.writers):
            batch.nov[w] = max(int(e0[a]), int(self.hi[a]))
        self.pending = batch
        return shard.ERR_OP_VERSION if self.flags & shard.SHARD_GAP else 0

    def dense_buffer(self):
        return torch.zeros(len(self.reg) + 2, dtype=torch.int64)

    def export_pending(self, dense):
        v = np.array([self.pending.state.get(a, 0) for a in self.reg], np.uint64)
        dense[: len(self.reg)] = torch.from_numpy(v.view(np.int64))
        return all(a in self.reg for a in self.pending.state)

    def commit(self, accept, reduced=None):
        p, self.pending = self.pending, None
        if not accept:
            return
        if reduced is not None:
            v = reduced.numpy().view(np.uint64)
            for i, a in enumerate(self.reg):
                if v[i]:
                    self.core.state[a] = max(self.core.state.get(a, 0), int(v[i]))
        else:
            for a, c in p.state.items():
                self.core.state[a] = max(self.core.state.get(a, 0), c)
        for a, c in p.nov.items():
            if c:
                self.core.nov[a] = max(self.core.nov.get(a, 0), c)
