"""Drop-in ``Oracle`` for the PCA consensus path, computed on MI355X.

Same constructor, attributes and ``consensus()`` result dict as the reference
``pyconsensus.Oracle`` (pyconsensus/__init__.py:100-611).  The host side only
normalises arguments and assembles the result containers; every number of the
result is computed by libpcx's HIP kernels:

* rounds with N <= 64 reporters and E <= 32 events run the one-wavefront round
  kernel (csrc/pcx_batched.hip) -- the same kernel as the batched Monte Carlo
  regime, with a batch of one;
* larger matrices run the single-matrix pipeline (one call of pcx_consensus_f64,
  csrc/pcx_runner.cpp + csrc/pcx_matrix.hip) on one GPU, or -- with
  ``devices=[0, 1, ...]`` -- row-sharded over several GPUs of this process
  (pcx_create_devices: one worker thread per GPU, RCCL over xGMI inside libpcx).

There is no CPU fallback: without the library or a GPU, ``consensus()`` raises.
"""
from __future__ import annotations

import time

import numpy as np

from . import _abi, _device
from .batched import MAX_EVENTS, MAX_REPORTERS, consensus_batched, unpack_round

NO, YES, BAD, NA = 1.0, 2.0, 1.5, 0.0  # __init__.py:65-68


class Oracle(object):
    """``Oracle(reports, event_bounds, reputation, ...).consensus()`` on the GPU.

    Supported ``algorithm`` values: ``"PCA"`` (default, the hot path), ``"big-five"``
    and ``"fixed-variance"`` (eigenvalue-weighted component scores, :373-390,
    :429-451), ``"cokurtosis"`` (``aux["cokurt"]`` scores, :455-457) and
    ``"absolute"`` (the reference's unimplemented branch: uniform this_rep,
    :359-362), and the clustering algorithms ``"k-means"`` (:392-405; its restarts draw
    from numpy's global RandomState exactly as the reference's scipy call does),
    ``"hierarchical"`` (:407-419) and ``"clusterfeck"`` (:148-242, :421-424): rounds of at
    most 64 reporters x 32 events on the batched kernel, larger matrices on the
    single-matrix path (one GPU).
    """

    def __init__(self, reports=None, event_bounds=None, reputation=None,
                 catch_tolerance=0.1, alpha=0.1, verbose=False,
                 aux=None, algorithm="PCA", variance_threshold=0.9,
                 max_components=5, hierarchy_threshold=0.5, device=None, devices=None):
        self.NO, self.YES, self.BAD, self.NA = NO, YES, BAD, NA
        data = np.ma.getdata(reports) if isinstance(reports, np.ma.MaskedArray) else reports
        arr = np.asarray(data)
        if arr.ndim != 2:
            raise ValueError("reports must be a 2-D reporters x events matrix")
        # Q2: a float ndarray is rescaled IN PLACE by the reference (:121, :269)
        self._caller = reports if (isinstance(reports, np.ndarray) and not isinstance(reports, np.ma.MaskedArray)
                                   and reports.dtype == np.float64) else None
        self._int_dtype = np.issubdtype(arr.dtype, np.integer)
        self._data = np.ascontiguousarray(arr, dtype=np.float64)
        self.reports = np.ma.masked_array(arr, np.isnan(arr.astype(np.float64)))
        self.num_reports, self.num_events = arr.shape
        self.event_bounds = event_bounds
        self.catch_tolerance = catch_tolerance
        self.alpha = alpha
        self.verbose = verbose
        self.algorithm = algorithm
        self.variance_threshold = variance_threshold
        self.num_components = -1
        self.hierarchy_threshold = hierarchy_threshold
        self.convergence = False
        self.aux = aux
        self.max_components = max_components if self.num_events >= max_components else self.num_events
        self.device = device
        # extension: shard the single-matrix path's rows over these GPUs (one process)
        self.devices = None if devices is None else [int(d) for d in devices]
        if self.devices is not None and not self.devices:
            raise ValueError("devices must list at least one GPU")
        n = self.num_reports
        if reputation is None:  # :138-141
            self.weighted = False
            self.total_rep = n
            self.reputation = np.array([1 / float(n)] * n)
            self._rep_raw = None
        else:  # :143-145 (the GPU recomputes these from the raw weights)
            self.weighted = True
            raw = np.asarray(reputation)
            self.total_rep = np.sum(raw.ravel())
            self.reputation = np.asarray(raw, dtype=np.float64).ravel() / float(self.total_rep)
            self._rep_raw = np.asarray(raw, dtype=np.float64).ravel()
        self.reptokens = [int(r * 1e6) for r in self.reputation]  # :146
        self.last_info = {}

    # -- scalar helpers of the reference API (:244-258) ------------------------
    def normalize(self, v):
        v = np.abs(v)
        if np.sum(v) == 0:
            v = v + 1
        return v / np.sum(v)

    def catch(self, X):
        if X < self.BAD - self.catch_tolerance:
            return self.NO
        elif X > self.BAD + self.catch_tolerance:
            return self.YES
        return self.BAD

    def _device_index(self):
        if self.devices is not None:
            return self.devices[0]
        if self.device is None:
            return 0
        import torch

        d = torch.device(self.device)
        return d.index or 0

    def _kw(self):
        return dict(catch_tolerance=self.catch_tolerance, alpha=self.alpha, algorithm=self._stage_algorithm(),
                    max_components=self.max_components, variance_threshold=self.variance_threshold,
                    devices=self.devices)

    def _stage_algorithm(self):
        return self.algorithm if self.algorithm in ("PCA", "absolute", "big-five", "fixed-variance",
                                                    "cokurtosis") else "PCA"

    # -- stage methods (:260-500), each one call of the single-matrix ABI ------
    def interpolate(self, reports):
        """Oracle.interpolate (:260-313): rescales the scaled events of ``reports`` IN PLACE
        (as the reference does, Q2) and returns the filled matrix (same dtype; an integer
        dtype truncates the fills, Q3).  Fills: weighted median (scaled) / catch of the
        weighted mean (binary), computed on the GPU (pcx_interpolate_f64)."""
        from .pipeline import interpolate_host

        data = np.ma.getdata(reports) if isinstance(reports, np.ma.MaskedArray) else np.asarray(reports)
        ints = np.issubdtype(data.dtype, np.integer)
        sc, lo, hi = self._bounds_arrays()
        outs, _ = interpolate_host(np.asarray(data, dtype=np.float64), self._rep_raw, sc, lo, hi,
                                   device_index=self._device_index(), int_dtype=ints, **self._kw())
        if sc is not None and sc.any():
            cols = np.nonzero(sc)[0]
            val = outs["original"][:, cols].astype(data.dtype) if ints else outs["original"][:, cols]
            if isinstance(reports, np.ma.MaskedArray):  # a masked column stays masked where NaN
                val = np.ma.masked_array(val, np.isnan(outs["original"][:, cols]))
            reports[:, cols] = val
        return outs["filled"].astype(data.dtype) if ints else outs["filled"]

    def wpca(self, reports_filled):
        """Oracle.wpca (:315-339) on the GPU (pcx_wpca_f64): returns (weighted_mean, wcd,
        covariance_matrix, first_loading, first_score).  The covariance is the token-weighted
        fp64-MFMA SYRK, the loading the power-iteration leading eigenvector (its sign follows
        the SPEC rule, which may differ from LAPACK's, Q8)."""
        from .pipeline import wpca_host

        F = np.asarray(np.ma.getdata(reports_filled), dtype=np.float64)
        outs, _ = wpca_host(F, self._rep_raw, device_index=self._device_index(), **self._kw())
        weighted_mean = np.ma.masked_array(outs["weighted_mean"])
        wcd = np.asmatrix(F - outs["weighted_mean"])
        first_loading = np.ma.masked_array(outs["adj_first_loadings"])
        first_score = np.asmatrix(outs["scores"])
        return weighted_mean, wcd, np.ma.masked_array(outs["covariance"]), first_loading, first_score

    def lie_detector(self, reports_filled):
        """Oracle.lie_detector (:341-473) on the GPU (pcx_lie_detector_f64): the algorithm's
        scores and sign choice, then this_rep / smooth_rep."""
        from .pipeline import lie_detector_host

        F = np.asarray(np.ma.getdata(reports_filled), dtype=np.float64)
        aux = None
        if self.algorithm == "cokurtosis":
            aux = np.asarray(self.aux["cokurt"], dtype=np.float64).ravel()
        kw = self._kw()
        if self.algorithm in _abi.CLUSTER_ALGORITHMS:
            # nc from the clusters (:392-424) on one GPU: the clusterings do not shard
            if self.devices is not None and len(set(self.devices)) > 1:
                raise NotImplementedError("the clustering algorithms run on one GPU; got devices=%r" % self.devices)
            kw.update(algorithm=self.algorithm, devices=None, hierarchy_threshold=self.hierarchy_threshold)
        elif self.algorithm not in _abi.ALGORITHMS:
            raise NotImplementedError("algorithm %r is not on the GPU path" % (self.algorithm,))
        outs, meta = lie_detector_host(F, self._rep_raw, device_index=self._device_index(), aux_scores=aux, **kw)
        self.convergence = self.algorithm != "absolute"
        if self.algorithm == "clusterfeck":  # cluster() rewrites zero tokens in the caller's list (:202-204)
            self.reptokens = [0.00001 if t == 0 else t for t in self.reptokens]
        self.last_info = {"branch": meta["branch"], "path": "matrix"}
        ma = np.ma.masked_array if self.algorithm == "PCA" else np.asarray
        return {"first_loading": np.ma.masked_array(outs["adj_first_loadings"]),
                "scores": ma(outs["scores"]) if aux is None else self.aux["cokurt"],
                "old_rep": self.reputation.T, "this_rep": ma(outs["this_rep"]),
                "smooth_rep": ma(outs["smooth_rep"])}

    def nonconformity(self, scores, reports):
        """Oracle.nonconformity (:475-485): the continuous sign choice, on the GPU."""
        return self._nonconformity(scores, reports, False)

    def nonconformity_rank(self, scores, reports):
        """Oracle.nonconformity_rank (:487-500): the rank rule with its continuous fallback."""
        return self._nonconformity(scores, reports, True)

    def _nonconformity(self, scores, reports, rank_rule):
        from .pipeline import nonconformity_host

        F = np.asarray(np.ma.getdata(reports), dtype=np.float64)
        s = np.asarray(np.ma.getdata(scores), dtype=np.float64).ravel()
        nc, meta = nonconformity_host(s, F, self._rep_raw, rank_rule=rank_rule,
                                      device_index=self._device_index(), **self._kw())
        self.convergence = True
        self.last_info = {"branch": meta["branch"], "path": "matrix"}
        return nc

    # -- consensus (:502-611) ---------------------------------------------------
    def _bounds_arrays(self):
        if self.event_bounds is None:
            return None, None, None
        sc = np.array([bool(b["scaled"]) for b in self.event_bounds], dtype=np.uint8)
        lo = np.array([float(b["min"]) for b in self.event_bounds], dtype=np.float64)
        hi = np.array([float(b["max"]) for b in self.event_bounds], dtype=np.float64)
        return sc, lo, hi

    def consensus(self):
        t0 = time.perf_counter()
        if self.algorithm not in _abi.ALGORITHMS:
            raise NotImplementedError("algorithm %r is not on the GPU path (supported: %s)"
                                      % (self.algorithm, ", ".join(sorted(_abi.ALGORITHMS))))
        sc, lo, hi = self._bounds_arrays()
        N, E = self.num_reports, self.num_events
        aux = None
        if self.algorithm == "cokurtosis":
            aux = np.asarray(self.aux["cokurt"], dtype=np.float64).ravel()  # :456
            if aux.size != N:
                raise ValueError("aux['cokurt'] must hold one score per reporter")
        kw = dict(catch_tolerance=self.catch_tolerance, alpha=self.alpha, int_dtype=self._int_dtype,
                  algorithm=self.algorithm, device=self.device if self.devices is None else self.devices[0],
                  max_components=self.max_components, variance_threshold=self.variance_threshold)
        small = N <= MAX_REPORTERS and E <= MAX_EVENTS
        t1 = time.perf_counter()
        if small:
            out = consensus_batched(self._data[None], None if self._rep_raw is None else self._rep_raw[None],
                                    sc, lo, hi, filled=True, original=True,
                                    aux_scores=None if aux is None else aux[None],
                                    hierarchy_threshold=self.hierarchy_threshold, packed=True, **kw)
            _device.synchronize(out["_packed"].device)  # (the device work apart from the copy back)
            t2 = time.perf_counter()
            g = unpack_round(out)
            t3 = time.perf_counter()
            participation = float(g["participation"])
            avg_certainty = float(g["avg_certainty"])
            comps = int(g["components"])
            self.last_info = {"branch": int(g["branch"]), "flags": int(g["flags"]),
                              "pi_iters": int(g["pi_iters"]), "path": "batched"}
        else:
            from .pipeline import consensus_host

            ckw = {}
            if self.algorithm in _abi.CLUSTER_ALGORITHMS:  # one GPU (the clusterings do not shard)
                ckw = dict(hierarchy_threshold=self.hierarchy_threshold)
            # Q2 without a host copy: when the caller's float64 array is the one the library reads,
            # `original` aliases it and libpcx rescales its scaled columns in place (else `original`
            # aliases this Oracle's own float64 copy)
            g, meta = consensus_host(self._data, self._rep_raw, sc, lo, hi, device_index=self._device_index(),
                                     aux_scores=aux, original_inplace=True,
                                     devices=None if self.algorithm in _abi.CLUSTER_ALGORITHMS else self.devices,
                                     **ckw, **{k: v for k, v in kw.items() if k != "device"})
            t2 = t3 = time.perf_counter()  # (one synchronous call: copies in, stages, copies out)
            participation = float(meta["participation"])
            avg_certainty = float(meta["avg_certainty"])
            comps = int(meta["components"])
            self.last_info = {"branch": meta["branch"], "flags": meta["flags"], "pi_iters": meta["pi_iters"],
                              "n_hard": meta["n_hard"], "sel_passes": meta["sel_passes"], "path": "matrix",
                              "devices": self.devices or [self._device_index()], "comm_bytes": meta["comm_bytes"],
                              "grid_events": meta["grid_events"], "mixed_int8": meta["mixed_int8"],
                              "cov_guard": meta["cov_guard"], "cov_guard_cols": meta["cov_guard_cols"],
                              "cov_err_bound": meta["cov_err_bound"]}
        if self.algorithm in ("big-five", "fixed-variance") and self.last_info["flags"] & _abi.FLAG_SVD_FAIL:
            # the reference's second svd (:375, :431) is outside the try of :329-333
            raise np.linalg.LinAlgError("SVD did not converge (non-finite covariance)")
        if self.algorithm == "fixed-variance":
            self.num_components = comps  # :449
        self.convergence = self.algorithm != "absolute"  # nonconformity(_rank) / the clusterings set it
        if self.algorithm == "clusterfeck":  # cluster() rewrites zero tokens in the caller's list (:202-204)
            self.reptokens = [0.00001 if t == 0 else t for t in self.reptokens]
        res = self._result(g, participation, avg_certainty)
        t4 = time.perf_counter()
        # per-call host timing (bench.py's c1 / c2 entries): argument preparation, the GPU call
        # (batched: inputs to the device, launch, kernel; matrix: the whole synchronous libpcx call),
        # the copy back (batched), and the result dict
        self.last_info["timing_ms"] = {"prepare": 1e3 * (t1 - t0), "gpu_call": 1e3 * (t2 - t1),
                                       "d2h": 1e3 * (t3 - t2), "assemble": 1e3 * (t4 - t3)}
        if self.verbose:
            self._print_verbose(res)
        return res

    def _print_verbose(self, res):
        """The reference's verbose=True trace (:349-357, :363-365, :463-466, :552-572),
        printed from the GPU results."""
        print("Reports:")
        print(self.reports)
        print("Total rep:")
        print(self.total_rep)
        print("Num reporters:")
        print(self.num_reports)
        print("Rep tokens:")
        print(self.reptokens)
        print("pyconsensus [%s]:\n" % self.algorithm)
        s = np.asarray(np.ma.getdata(res["agents"]["scores"]), dtype=np.float64)
        b = self.last_info.get("branch", _abi.BRANCH_NONE)
        if b in (_abi.BRANCH_SET1, _abi.BRANCH_TIE_SET1):
            nc = s + np.abs(np.min(s))
        elif b in (_abi.BRANCH_SET2, _abi.BRANCH_TIE_SET2):
            nc = s - np.max(s)
        else:
            nc = np.zeros(self.num_reports)
        print("  Adjusted:  ", nc)
        print("  Reputation:", res["agents"]["this_rep"])
        print()
        na = np.ma.masked_array(np.asarray(res["agents"]["na_row"]))
        print("NA Mat:")
        print(np.isnan(np.ma.getdata(self.reports).astype(np.float64)) | (np.ma.getdata(self.reports) == NA))
        print()
        print("Sum:")
        print(na)
        print()
        print(1 - res["participation"])

    def _result(self, g, participation, avg_certainty):
        original = g["original"]
        filled = g["filled"]
        if self._int_dtype:  # int64 storage truncates (Q3)
            original = original.astype(np.int64)
            filled = filled.astype(np.int64)
        if self._caller is not None and not np.shares_memory(self._caller, g["original"]):
            self._caller[...] = g["original"]  # Q2: the caller's float array carries the rescaled values
        self.reports = np.ma.masked_array(original, self.reports.mask)
        ints = self._int_dtype
        cnt = (lambda a: [int(x) for x in a]) if ints else (lambda a: [float(x) for x in a])
        # PCA's reputation vectors and scores are MaskedArrays (the masked first loading
        # propagates, :336-337); the other algorithms produce plain ndarrays
        ma = np.ma.masked_array if self.algorithm == "PCA" else np.asarray
        scores = g["scores"]
        if self.algorithm == "cokurtosis":
            scores = self.aux["cokurt"]  # returned as given (:457)
        outcomes_adj = [float(x) for x in g["outcomes_adjusted"]]
        return {
            "original": original,
            "filled": filled,
            "agents": {
                "old_rep": g["old_rep"],
                "this_rep": ma(g["this_rep"]),
                "smooth_rep": ma(g["smooth_rep"]),
                "na_row": cnt(g["na_row"]),
                "participation_rows": [float(x) for x in g["participation_rows"]],
                "relative_part": [float(x) for x in g["relative_part"]],
                "reporter_bonus": [float(x) for x in g["reporter_bonus"]],
                "scores": ma(scores) if self.algorithm != "cokurtosis" else scores,
            },
            "events": {
                "adj_first_loadings": [float(x) for x in g["adj_first_loadings"]],
                "outcomes_raw": [float(x) for x in g["outcomes_raw"]],
                "consensus_reward": g["consensus_reward"],
                "certainty": g["certainty"],
                "NAs Filled": cnt(g["nas_filled"]),
                "participation_columns": [float(x) for x in g["participation_columns"]],
                "author_bonus": [float(x) for x in g["author_bonus"]],
                "outcomes_adjusted": outcomes_adj,
                "outcomes_final": [float(x) for x in g["outcomes_final"]],
            },
            "participation": participation,
            "avg_certainty": avg_certainty,
            "convergence": self.convergence,
            "components": self.num_components,
        }
