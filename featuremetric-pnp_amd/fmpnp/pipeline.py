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
placement differs).

`window=r` (the f-only layout) packs only the texels within r texels of each point's texel
at the initial pose (fmpnp_pack_features_f_window_batch): the refinement reads only the 3x3
neighbourhoods of the texels its points visit, a few texels from where they start.  The LM
kernel checks every gather against the window and stops a problem that leaves it
(FMPNP_STATUS_WINDOW); such queries are packed in full and refined again, so every result
equals the fully packed pipeline's bit for bit.

`levels=[(c_begin, c_end), ...]` runs multilevel_optimization's channel pyramid
(featurePnP/model.py:178-213, e.g. input_configs/default_robotcar.gin:75) on each batch: one LM
launch per level over channel slices of the same packed map, each level starting from the
previous level's poses, copied result -> descriptor on the device (no host round trip).  A query is (query_hc [C,H,W] or [1,C,H,W] device tensor,
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


class _LevelChain:
    """One batch's LM launches over the channel levels: level l > 0 takes its initial poses from
    level l - 1's results (R, t -> R0, t0 of the device descriptors) on the launching stream."""

    def __init__(self, batches):
        self.levels = batches
        self.d_descs = batches[0].d_descs
        self.d_res = batches[-1].d_res
        self.d_ws = batches[0].d_ws

    def launch(self, stream=None):
        rs, ps = _rf.RESULT_DTYPE.itemsize, _rf.PROBLEM_DTYPE.itemsize
        o_res, o_prob = _rf.RESULT_DTYPE.fields["R"][1], _rf.PROBLEM_DTYPE.fields["R0"][1]
        for li, b in enumerate(self.levels):
            if li:  # (R[9], t[3] and R0[9], t0[3] are contiguous: one 96-byte copy per problem)
                prev = self.levels[li - 1].d_res.view(b.n, rs)
                b.d_descs.view(b.n, ps)[:, o_prob:o_prob + 96].copy_(prev[:, o_res:o_res + 96], non_blocking=True)
            b.launch(stream)

    def tensors(self):
        return [t for b in self.levels for t in (b.d_descs, b.d_res, b.d_ws)]

    def results(self):
        """The last level's results; every level's status in `level_status`, and the bits that say
        an earlier level went wrong ORed in: a timed-out exchange (its poses unrefined) and a NaN
        step (model.py:411-413) -- both seed the next level with a pose that was not refined."""
        res = self.levels[-1].results()
        earlier = [b.results() for b in self.levels[:-1]]
        for q, r in enumerate(res):
            r["level_status"] = [e[q]["status"] for e in earlier] + [r["status"]]
            for e in earlier:
                r["status"] |= e[q]["status"] & (_lib.STATUS_SYNC_TIMEOUT | _lib.STATUS_NAN)
        return res


def _streams(device):
    if device.index not in _STREAMS:
        _STREAMS[device.index] = (torch.cuda.Stream(device), torch.cuda.Stream(device))
    return _STREAMS[device.index]


class RefinePipeline:
    def __init__(self, image_shape=None, storage=torch.float32, device=None, depth=2, model_kwargs=None,
                 sampling="nearest", layout=None, wgs_per_problem=None, window=None, levels=None):
        cfg = config.adapter_kwargs()
        self.image_shape = tuple(image_shape or cfg.get("image_shape", (1024, 1024)))
        self.storage = storage
        self.device = torch.device(device) if device is not None else torch.device("cuda", torch.cuda.current_device())
        _lib.require_device(self.device)
        kw = config.model_kwargs()
        kw.update(model_kwargs or {})
        loss_code, alpha = _losses.resolve(kw["loss_fn"])
        # workgroups per query (None: per batch, as many as keep the LM launch on half of the CUs,
        # the other half left to the next batch's pack and gather on the prep stream -- RobotCar
        # C = 1664, 32 queries: G = 4 3.84 k queries/s against G = 1 3.34 k and the planner's G = 8
        # 3.64 k, tools/robotcar_e2e.py), and no first-evaluation helpers: no workgroup of a launch
        # waits on another one (a helper) that those concurrent kernels could keep from being resident
        self.wgs = None if wgs_per_problem is None else int(wgs_per_problem)
        self.ncu = torch.cuda.get_device_properties(self.device).multi_processor_count
        self.options = _rf.make_options(kw["n_iters"], kw["lambda_"], loss_code, alpha, kw.get("ratio_threshold"),
                                        _rf._dtype_code(storage), sampling=sampling,
                                        wgs_per_problem=self.wgs or 0, helpers=-1)
        self.sampling = sampling
        self.depth = max(1, int(depth))
        # "f" (f plane only, gradients formed in the LM gather) wherever it applies: fp32
        # texels, nearest sampling; "fgrad" (the packed f, gx, gy planes) otherwise
        f_ok = storage == torch.float32 and sampling == "nearest"
        self.layout = layout or ("f" if f_ok else "fgrad")
        if self.layout == "f" and not f_ok:
            raise ValueError("layout 'f' needs fp32 storage and nearest sampling")
        self.window = None if window is None else int(window)
        if self.window is not None and (self.layout != "f" or self.window < 2):
            raise ValueError("window needs the f-only layout and a radius >= 2")
        self.refills = 0  # queries re-run with the full pack after leaving their window
        # host seconds (perf_counter) in preparing batches (of which the first batch's: nothing
        # runs on the device yet), collecting results while streaming, and the final drain
        self.host_s = {"prepare": 0.0, "first_prepare": 0.0, "finish": 0.0, "drain": 0.0}
        self.unwindowed_batches = 0  # batches packed in full: a problem too large for a windowed plan
        self.levels = [tuple(int(c) for c in lv) for lv in levels] if levels else None
        if self.levels and self.window is not None:
            raise ValueError("channel levels run on fully packed maps (window=None)")
        self.bound_options = _lib.Options.from_buffer_copy(self.options)
        self.bound_options.layout = _lib.LAYOUT_F if self.layout == "f" else _lib.LAYOUT_FGRAD
        self.prep, self.solve = _streams(self.device)
        self.slabs = [None] * self.depth        # flat uint8 device buffers holding a batch's packed maps
        self.slab_free = [None] * self.depth    # event: the last launch that read the slab finished

    def batch_options(self, nq):
        """The launch options of a batch of nq queries: the bound options with the batch's
        workgroups per query (a packed window takes one, fmpnp_api.hip make_plan)."""
        o = _lib.Options.from_buffer_copy(self.bound_options)
        o.wgs_per_problem = self.wgs if self.wgs is not None else max(1, (self.ncu // 2) // max(nq, 1))
        return o

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
        C-ABI call each for the packs and the reference gathers, and the LM descriptors
        filled column-wise (no per-query host objects)."""
        dev, storage = self.device, self.storage
        nq = len(queries)
        qmaps = [q if q.dim() == 3 else q[0] for (q, _, _, _) in queries]
        rmaps = [r if r.dim() == 3 else r[0] for (_, r, _, _) in queries]
        q_dt = qmaps[0].dtype if qmaps[0].dtype in (torch.float32, torch.float64) else torch.float32
        r_dt = rmaps[0].dtype if rmaps[0].dtype in (torch.float32, torch.float64) else torch.float32
        es = 4 if storage == torch.float32 else 8
        planes = 3 if self.layout == "fgrad" else 1
        Cs = np.array([m.shape[0] for m in qmaps], dtype=np.int64)
        Hs = np.array([m.shape[1] for m in qmaps], dtype=np.int64)
        Ws = np.array([m.shape[2] for m in qmaps], dtype=np.int64)
        css = (Cs + 3) // 4 * 4
        sizes = Hs * Ws * planes * css * es
        if self.window is not None:  # [2][H][W] window bytes after each map
            sizes = (sizes + _ALIGN - 1) // _ALIGN * _ALIGN + 2 * Hs * Ws
        starts = np.concatenate([[0], np.cumsum((sizes + _ALIGN - 1) // _ALIGN * _ALIGN)])
        inl = [np.asarray(q[2].reference_inliers, np.float64).reshape(-1, 2) for q in queries]
        pts = [np.asarray(q[2].points_3d, np.float64).reshape(-1, 3) for q in queries]
        n_pts = np.array([a.shape[0] for a in inl], dtype=np.int64)
        fr_off = np.concatenate([[0], np.cumsum(n_pts * css)])
        # the caller produced the hypercolumns on its own (current) stream: the prep stream
        # must not read them before that work finished
        self.prep.wait_stream(torch.cuda.current_stream(dev))
        for m in qmaps + rmaps:
            if m.is_cuda:
                m.record_stream(self.prep)
        with torch.cuda.device(dev), torch.cuda.stream(self.prep):
            def ready(m, dt):  # device, batch dtype, contiguous (else one conversion copy)
                return m if (m.is_cuda and m.dtype == dt and m.is_contiguous()) else _rf._as_device(m, dev, dt)
            qmaps = [ready(m, q_dt) for m in qmaps]
            rmaps = [ready(m, r_dt) for m in rmaps]
            slab = self._slab(k, max(int(starts[-1]), 1))
            out_ptrs = slab.data_ptr() + starts[:-1]
            if planes == 3 and (css != Cs).any():  # the Sobel pack writes channels < C only
                for i in np.nonzero(css != Cs)[0]:
                    slab[int(starts[i]):int(starts[i] + sizes[i])].zero_()
            # one out-of-map flag per query, read once the batch finished (no host wait here)
            err = torch.zeros(nq, dtype=torch.int32, device=dev)
            # every query's reference inliers and 3D points in one pinned upload (written straight into
            # pinned memory: one host copy)
            offs = np.concatenate([[0], np.cumsum([a.size for a in inl + pts])])
            pinned = torch.empty(int(offs[-1]), dtype=torch.float64, pin_memory=True)
            np.concatenate([a.reshape(-1) for a in inl + pts], out=pinned.numpy())
            dflat = pinned.to(dev, non_blocking=True)
            # reference descriptors of the whole batch: [N_i][cstride_i] runs in one buffer
            pad = any(int(css[i]) != rmaps[i].shape[0] for i in range(nq))
            fbuf = (torch.zeros if pad else torch.empty)(max(int(fr_off[-1]), 1), dtype=storage, device=dev)
            fr_ptrs = fbuf.data_ptr() + es * fr_off[:-1]
            L = _lib.load()
            vp = ctypes.c_void_p
            s = _lib.stream_ptr(dev)
            shape_arr = (ctypes.c_int * (4 * nq))(*np.stack([Cs, Hs, Ws, css], 1).reshape(-1).tolist())
            if self.window is None:
                rc = L.fmpnp_pack_features_batch(
                    nq, (vp * nq)(*[m.data_ptr() for m in qmaps]), (vp * nq)(*out_ptrs.tolist()), shape_arr,
                    _rf._dtype_code(q_dt), _rf._dtype_code(storage), 0, 0,
                    _lib.LAYOUT_F if self.layout == "f" else _lib.LAYOUT_FGRAD, s)            # :57, :61
                _lib.check(rc, "fmpnp_pack_features_batch")
            rshape = (ctypes.c_int * (3 * nq))(*[v for m in rmaps for v in m.shape])
            base = dflat.data_ptr()
            rc = L.fmpnp_gather_reference_batch(
                nq, (vp * nq)(*[m.data_ptr() for m in rmaps]), rshape, (vp * nq)(*(base + 8 * offs[:nq]).tolist()),
                (ctypes.c_int * nq)(*n_pts.tolist()), int(self.image_shape[0]), int(self.image_shape[1]),
                (vp * nq)(*fr_ptrs.tolist()), (ctypes.c_int * nq)(*css.tolist()), _rf._dtype_code(r_dt),
                _rf._dtype_code(storage), vp(err.data_ptr()), s)                               # :51-56
            _lib.check(rc, "fmpnp_gather_reference_batch")
            # LM descriptors, column by column (fmpnp_problem)
            desc = np.zeros(nq, dtype=_rf.PROBLEM_DTYPE)
            desc["feat"], desc["fref"], desc["pts3d"] = out_ptrs, fr_ptrs, base + 8 * offs[nq:2 * nq]
            desc["Hf"], desc["Wf"], desc["cstride"] = Hs, Ws, css
            desc["c_end"], desc["ld_ref"], desc["N"] = Cs, css, n_pts
            desc["im_width"], desc["im_height"] = int(self.image_shape[0]), int(self.image_shape[1])   # :52
            T = np.stack([np.asarray(q[2].matrix, np.float64) for q in queries])                    # :59-60
            desc["K"] = np.stack([np.asarray(q[3], np.float64).reshape(9) for q in queries])
            desc["R0"] = T[:, :3, :3].reshape(nq, 9)
            desc["t0"] = T[:, :3, 3]
            if self.window is not None:
                desc["window"] = out_ptrs + (Hs * Ws * css * es + _ALIGN - 1) // _ALIGN * _ALIGN
            opts = self.batch_options(nq)
            windowed = self.window is not None and self._window_fits(desc, opts)
            if self.window is not None and not windowed:
                # a packed window takes one workgroup per problem; a problem too large for one
                # workgroup's LDS (fmpnp_api.hip make_plan: ETOOBIG) gets this batch fully packed
                desc["window"] = 0
                self.unwindowed_batches += 1
                rc = L.fmpnp_pack_features_batch(
                    nq, (vp * nq)(*[m.data_ptr() for m in qmaps]), (vp * nq)(*out_ptrs.tolist()), shape_arr,
                    _rf._dtype_code(q_dt), _rf._dtype_code(storage), 0, 0, _lib.LAYOUT_F, s)
                _lib.check(rc, "fmpnp_pack_features_batch")
            if self.levels:
                chain = []
                for cb, ce in self.levels:
                    if not (0 <= cb < ce <= int(Cs.min())):
                        raise ValueError(f"channel level ({cb}, {ce}) outside the maps' {int(Cs.min())} channels")
                    dl = desc.copy()
                    dl["c_begin"], dl["c_end"] = cb, ce
                    chain.append(_rf.AsyncBatch.from_descriptors(dl, opts, dev, non_blocking=True))
                batch = _LevelChain(chain)
            else:
                batch = _rf.AsyncBatch.from_descriptors(desc, opts, dev, non_blocking=True)
            if windowed:  # the windowed pack reads the uploaded descriptors
                rc = L.fmpnp_pack_features_f_window_batch(
                    vp(batch.d_descs.data_ptr()), vp(batch.descs_np.ctypes.data), nq, (vp * nq)(*[m.data_ptr() for m in qmaps]),
                    _rf._dtype_code(q_dt), self.window, s)                                     # :57, :61
                _lib.check(rc, "fmpnp_pack_features_f_window_batch")
        # read on the prep stream (maps, converted copies) or the solve stream (the rest):
        # kept alive until the batch is collected
        return batch, [qmaps, rmaps, fbuf, dflat, desc], err

    def _window_fits(self, desc, opts):
        """Whether the batch's windowed launch plan exists (one workgroup per problem must hold
        the largest problem in its LDS)."""
        d = desc.copy()
        d["window"] = 1 << 12  # (any non-null pointer: the plan reads sizes only)
        return _lib.load().fmpnp_workspace_size(d.ctypes.data_as(ctypes.POINTER(_lib.Problem)), len(d),
                                                ctypes.byref(opts)) != 0

    def _refill(self, res, keep):
        """Queries that left their packed window: pack their maps in full and refine them again
        (same kernel, same descriptors but the window and the packed map)."""
        bad = [i for i, r in enumerate(res) if r["status"] & _lib.STATUS_WINDOW]
        if not bad:
            return res
        qmaps, desc = keep[0], keep[4]
        dev = self.device
        sub = desc[bad].copy()
        sub["window"] = 0
        bufs = []
        L = _lib.load()
        with torch.cuda.device(dev), torch.cuda.stream(self.solve):
            for j, i in enumerate(bad):
                m = qmaps[i]
                C, H, W = m.shape
                cs = int(sub["cstride"][j])
                buf = torch.empty(H * W * cs, dtype=torch.float32, device=dev)
                bufs.append(buf)
                rc = L.fmpnp_pack_features_f(ctypes.c_void_p(m.data_ptr()), _rf._dtype_code(m.dtype), C, H, W,
                                             ctypes.c_void_p(buf.data_ptr()), _lib.F32, cs, _lib.stream_ptr(dev))
                _lib.check(rc, "fmpnp_pack_features_f")
                sub["feat"][j] = buf.data_ptr()
            b = _rf.AsyncBatch.from_descriptors(sub, self.batch_options(len(bad)), dev)
            b.launch(_lib.stream_ptr(dev))
            again = b.results()
        self.refills += len(bad)
        res = list(res)
        for j, i in enumerate(bad):
            res[i] = again[j]
        return res

    def run(self, batches):
        """batches: iterable of lists of queries.  Returns a list (per batch) of result dicts
        (see refine.refine), computed with preparation and refinement overlapped."""
        inflight = []   # (batch, keep-alive buffers, err flags, done event) in submission order
        out = []

        def finish(entry):
            b, _, err, ev = entry
            ev.synchronize()
            bad = torch.nonzero(err.cpu()).flatten().tolist()
            if bad:
                raise IndexError(f"batch {len(out)}: reference inliers of queries {bad} map outside the reference "
                                 "hypercolumn (optimize_feature_pnp.py:56 raises IndexError)")
            res = b.results()
            if self.window is not None:
                res = self._refill(res, entry[1])
            # as refine.refine(): a timed-out cross-workgroup exchange left poses unrefined
            if any(r["status"] & _lib.STATUS_SYNC_TIMEOUT for r in res):
                raise _lib.FmpnpError(f"batch {len(out)}: cross-workgroup exchange timed out")
            out.append(res)

        import time
        for i, queries in enumerate(batches):
            # the host stays at most `depth` batches ahead of the collected results
            while len(inflight) >= self.depth:
                t0 = time.perf_counter()
                finish(inflight.pop(0))
                self.host_s["finish"] += time.perf_counter() - t0
            k = i % self.depth
            t0 = time.perf_counter()
            batch, keep, err = self._prepare(list(queries), k)
            self.host_s["prepare"] += time.perf_counter() - t0
            if i == 0:
                self.host_s["first_prepare"] += time.perf_counter() - t0
            ready = torch.cuda.Event()
            ready.record(self.prep)
            self.solve.wait_event(ready)
            with torch.cuda.device(self.device), torch.cuda.stream(self.solve):
                batch.launch(_lib.stream_ptr(self.device))
                # buffers written on the prep stream and read on the solve stream
                extra = batch.tensors() if isinstance(batch, _LevelChain) else [batch.d_descs, batch.d_res, batch.d_ws]
                for t in extra + [err, self.slabs[k], keep[2], keep[3]]:
                    t.record_stream(self.solve)
            done = torch.cuda.Event()
            done.record(self.solve)
            self.slab_free[k] = done
            inflight.append((batch, keep, err, done))
            del batch, keep, err
        t0 = time.perf_counter()
        for entry in inflight:
            finish(entry)
        self.host_s["drain"] += time.perf_counter() - t0
        return out
