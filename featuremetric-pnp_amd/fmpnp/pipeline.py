"""Streamed batch refinement: feature preparation of batch i+1 overlaps the LM launch of
batch i on a second HIP stream.

The per-query preparation of `feature_pnp` (optimize_feature_pnp.py:50-71 -> the fused
Sobel + channels-last pack and the reference-descriptor gather) streams every query's
hypercolumn through HBM once -- bandwidth-bound -- while the LM launch over a batch is
latency-bound and reads little.  `RefinePipeline` runs the preparation on a `prep`
stream and the LM launches on a `solve` stream, ordered by events:

  * the packed maps of a batch live in one of `depth` slabs (a ring, reused across
    batches and grown only when a batch needs more); the prep stream waits on the
    event of the launch that last read a slab before packing into it again, so slab
    reuse never blocks the host;
  * every query's reference inliers and 3D points go up in one pinned, asynchronous
    copy; out-of-map inliers (the reference's IndexError, optimize_feature_pnp.py:56)
    set a per-query device flag that is checked when the batch's results are read,
    so preparing a batch never waits for the device;
  * the host runs at most `depth` batches ahead of the results it has collected.

Results equal launching every batch alone (same kernels, same inputs; only the stream
placement differs).  A query is (query_hc [C,H,W] or [1,C,H,W] device tensor,
reference_hc, prediction, K) with the reference's `Prediction` fields (points_3d,
reference_inliers, matrix).
"""
import ctypes

import numpy as np
import torch

from . import _lib, config
from . import losses as _losses
from . import refine as _rf

_ALIGN = 256          # byte alignment of each packed map inside a slab
_STREAMS = {}         # device index -> (prep, solve): shared so the allocator's per-stream pools are reused


def _streams(device):
    if device.index not in _STREAMS:
        _STREAMS[device.index] = (torch.cuda.Stream(device), torch.cuda.Stream(device))
    return _STREAMS[device.index]


class RefinePipeline:
    def __init__(self, image_shape=None, storage=torch.float32, device=None, depth=2, model_kwargs=None,
                 sampling="nearest", layout=None):
        cfg = config.adapter_kwargs()
        self.image_shape = tuple(image_shape or cfg.get("image_shape", (1024, 1024)))
        self.storage = storage
        self.device = torch.device(device) if device is not None else torch.device("cuda", torch.cuda.current_device())
        _lib.require_device(self.device)
        kw = config.model_kwargs()
        kw.update(model_kwargs or {})
        loss_code, alpha = _losses.resolve(kw["loss_fn"])
        self.options = _rf.make_options(kw["n_iters"], kw["lambda_"], loss_code, alpha, kw.get("ratio_threshold"),
                                        _rf._dtype_code(storage), sampling=sampling)
        self.depth = max(1, int(depth))
        # "f" (f plane only, gradients formed in the LM gather) wherever it applies: fp32
        # texels, nearest sampling; "fgrad" (the packed f, gx, gy planes) otherwise
        f_ok = storage == torch.float32 and sampling == "nearest"
        self.layout = layout or ("f" if f_ok else "fgrad")
        if self.layout == "f" and not f_ok:
            raise ValueError("layout 'f' needs fp32 storage and nearest sampling")
        self.prep, self.solve = _streams(self.device)
        self.slabs = [None] * self.depth        # flat uint8 device buffers holding a batch's packed maps
        self.slab_free = [None] * self.depth    # event: the last launch that read the slab finished

    def _slab(self, k, nbytes):
        """Slab k with room for nbytes, usable on the prep stream once its last reader finished."""
        if self.slab_free[k] is not None:
            self.prep.wait_event(self.slab_free[k])
        if self.slabs[k] is None or self.slabs[k].numel() < nbytes:
            self.slabs[k] = None
            with torch.cuda.stream(self.prep):
                self.slabs[k] = torch.empty(nbytes, dtype=torch.uint8, device=self.device)
        return self.slabs[k]

    def _prepare(self, queries, k):
        """Pack + gather every query of a batch on the prep stream into slab k: one batched
        C-ABI call each for the Sobel packs and the reference gathers (no per-query host
        round trips)."""
        dev, storage = self.device, self.storage
        nq = len(queries)
        qmaps = [q if q.dim() == 3 else q[0] for (q, _, _, _) in queries]
        rmaps = [r if r.dim() == 3 else r[0] for (_, r, _, _) in queries]
        q_dt = qmaps[0].dtype if qmaps and qmaps[0].dtype in (torch.float32, torch.float64) else torch.float32
        r_dt = rmaps[0].dtype if rmaps and rmaps[0].dtype in (torch.float32, torch.float64) else torch.float32
        es = torch.empty(0, dtype=storage).element_size()
        planes = 3 if self.layout == "fgrad" else 1
        shapes = [(m.shape[1], m.shape[2], planes, _rf._round4(m.shape[0])) for m in qmaps]
        sizes = [int(np.prod(sh)) * es for sh in shapes]
        starts = np.concatenate([[0], np.cumsum([(b + _ALIGN - 1) // _ALIGN * _ALIGN for b in sizes])]).astype(int)
        inl = [np.asarray(p.reference_inliers, np.float64).reshape(-1, 2) for (_, _, p, _) in queries]
        pts = [np.asarray(p.points_3d, np.float64).reshape(-1, 3) for (_, _, p, _) in queries]
        n_pts = [a.shape[0] for a in inl]
        probs = []
        with torch.cuda.device(dev), torch.cuda.stream(self.prep):
            qmaps = [_rf._as_device(m, dev, q_dt) for m in qmaps]   # no-ops for device maps of the batch dtype
            rmaps = [_rf._as_device(m, dev, r_dt) for m in rmaps]
            slab = self._slab(k, max(int(starts[-1]), 1))
            outs = [slab[starts[i]:starts[i] + sizes[i]].view(storage).view(shapes[i] if planes == 3 else
                                                                              (shapes[i][0], shapes[i][1],
                                                                               shapes[i][3]))
                    for i in range(nq)]
            for i in range(nq):
                if shapes[i][3] != qmaps[i].shape[0]:
                    outs[i].zero_()  # padding channels stay zero (the kernel writes c < C only)
            # one out-of-map flag per query, read once the batch finished (no host wait here)
            err = torch.zeros(nq, dtype=torch.int32, device=dev)
            # every query's reference inliers and 3D points in one pinned upload
            flat = np.concatenate([a.reshape(-1) for a in inl + pts]) if nq else np.zeros(0)
            dflat = torch.from_numpy(flat).pin_memory().to(dev, non_blocking=True)
            offs = np.concatenate([[0], np.cumsum([a.size for a in inl + pts])]).astype(int)
            # reference descriptors of the whole batch: [N_i][cstride_i] runs in one buffer
            fr_off = np.concatenate([[0], np.cumsum([n_pts[i] * shapes[i][3] for i in range(nq)])]).astype(int)
            pad = any(shapes[i][3] != rmaps[i].shape[0] for i in range(nq))
            fbuf = (torch.zeros if pad else torch.empty)(max(int(fr_off[-1]), 1), dtype=storage, device=dev)
            frefs = [fbuf[fr_off[i]:fr_off[i + 1]].view(n_pts[i], shapes[i][3]) for i in range(nq)]
            L = _lib.load()
            vp = ctypes.c_void_p
            s = _lib.stream_ptr(dev)
            shape_arr = (ctypes.c_int * (4 * nq))(*[v for i in range(nq) for v in
                                                    (qmaps[i].shape[0], shapes[i][0], shapes[i][1], shapes[i][3])])
            rc = L.fmpnp_pack_features_batch(
                nq, (vp * nq)(*[m.data_ptr() for m in qmaps]), (vp * nq)(*[o.data_ptr() for o in outs]), shape_arr,
                _rf._dtype_code(q_dt), _rf._dtype_code(storage), 0, 0,
                _lib.LAYOUT_F if self.layout == "f" else _lib.LAYOUT_FGRAD, s)                # :57, :61
            _lib.check(rc, "fmpnp_pack_features_batch")
            rshape = (ctypes.c_int * (3 * nq))(*[v for m in rmaps for v in m.shape])
            base = dflat.data_ptr()
            rc = L.fmpnp_gather_reference_batch(
                nq, (vp * nq)(*[m.data_ptr() for m in rmaps]), rshape,
                (vp * nq)(*[base + 8 * int(offs[i]) for i in range(nq)]), (ctypes.c_int * nq)(*n_pts),
                int(self.image_shape[0]), int(self.image_shape[1]), (vp * nq)(*[f.data_ptr() for f in frefs]),
                (ctypes.c_int * nq)(*[sh[3] for sh in shapes]), _rf._dtype_code(r_dt), _rf._dtype_code(storage),
                vp(err.data_ptr()), s)                                                        # :51-56
            _lib.check(rc, "fmpnp_gather_reference_batch")
            for i, (_, _, pred, K) in enumerate(queries):
                feats = _rf.PackedFeatures(outs[i], qmaps[i].shape[0], shapes[i][0], shapes[i][1], shapes[i][3],
                                           self.layout, 0)
                T = np.asarray(pred.matrix, dtype=np.float64)
                probs.append(_rf.make_problem(feats, frefs[i], dflat[offs[nq + i]:offs[nq + i + 1]].view(-1, 3),
                                              np.asarray(K, np.float64).reshape(3, 3), self.image_shape[0],
                                              self.image_shape[1], T[:3, :3], T[:3, 3]))     # :52, :59-60
            batch = _rf.AsyncBatch(probs, self.options, non_blocking=True)
        # the maps are read on the prep stream only; keep them (and any converted copies)
        # alive until the batch is collected
        return batch, probs + [qmaps, rmaps, fbuf], err

    def run(self, batches):
        """batches: iterable of lists of queries.  Returns a list (per batch) of result dicts
        (see refine.refine), computed with preparation and refinement overlapped."""
        inflight = []   # (batch, probs, err flags, done event) in submission order
        out = []

        def finish(entry):
            b, _, err, ev = entry
            ev.synchronize()
            bad = torch.nonzero(err.cpu()).flatten().tolist()
            if bad:
                raise IndexError(f"batch {len(out)}: reference inliers of queries {bad} map outside the reference "
                                 "hypercolumn (optimize_feature_pnp.py:56 raises IndexError)")
            out.append(b.results())

        for i, queries in enumerate(batches):
            # the host stays at most `depth` batches ahead of the collected results
            while len(inflight) >= self.depth:
                finish(inflight.pop(0))
            k = i % self.depth
            batch, probs, err = self._prepare(list(queries), k)
            ready = torch.cuda.Event()
            ready.record(self.prep)
            self.solve.wait_event(ready)
            with torch.cuda.device(self.device), torch.cuda.stream(self.solve):
                batch.launch(_lib.stream_ptr(self.device))
                # buffers written on the prep stream and read on the solve stream
                for p in probs:
                    if isinstance(p, _rf.Problem):
                        p.fref.record_stream(self.solve)
                        p.pts3d.record_stream(self.solve)
                for t in (batch.d_descs, batch.d_res, batch.d_ws, err, self.slabs[k]):
                    t.record_stream(self.solve)
            done = torch.cuda.Event()
            done.record(self.solve)
            self.slab_free[k] = done
            inflight.append((batch, probs, err, done))
            del batch, probs, err
        for entry in inflight:
            finish(entry)
        return out
