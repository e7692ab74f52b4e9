"""Thin torch-tensor wrappers over the C ABI (include/mapfed.h).

torch supplies device memory and the current HIP stream; every compute call goes through
libmapfed.so.  Wrappers allocate outputs only when the caller passes none (the engine always
passes preallocated buffers so a whole step can be captured in a hipGraph).
"""
from __future__ import annotations

import ctypes
import os
from typing import Optional

import torch

from ._lib import call

EPI_NONE, EPI_BIAS, EPI_BIAS_RESID, EPI_BIAS_GELU, EPI_DGELU, EPI_F32, EPI_RESID = range(7)


class KernelProbe:
    """Brackets every launch of the probed kernel families with HIP events on the launching stream
    (used by bench.py for the per-launch rooflines; off by default, never active during graph
    capture).  kinds: "gemm", "attention" (or one name / an iterable); each record carries a key
    ("gemm", "attention_fwd/L199", ...) so the families and towers are summarised separately."""

    def __init__(self, kinds="gemm"):
        self.kinds = {kinds} if isinstance(kinds, str) else set(kinds)
        self.kind = next(iter(self.kinds)) if len(self.kinds) == 1 else None  # single-family callers
        self.records = []  # (key, start_event, end_event, flops, bytes, meta)

    def wants(self, kind: str) -> bool:
        return kind in self.kinds

    def around(self, flops: float, nbytes: float, key: str = "gemm", meta=None):
        """meta: what the launch was (the GEMMs: (M, N, K, epilogue)), for per-shape tables."""
        s = torch.cuda.Event(enable_timing=True)
        e = torch.cuda.Event(enable_timing=True)
        s.record()
        self.records.append((key, s, e, flops, nbytes, meta))
        return e

    def launches(self):
        """Per-launch records in launch order: key, duration (us), flops, algorithmic bytes, meta."""
        torch.cuda.synchronize()
        return [{"key": k, "us": 1e3 * s.elapsed_time(e), "flops": f, "bytes": b, "meta": m}
                for k, s, e, f, b, m in self.records]

    def keys(self):
        return sorted({r[0] for r in self.records})

    def summary(self, prefix: Optional[str] = None):
        torch.cuda.synchronize()
        recs = [r for r in self.records if prefix is None or r[0].startswith(prefix)]
        ms = [r[1].elapsed_time(r[2]) for r in recs]
        n = len(ms)
        tot_ms = sum(ms)
        flops = sum(r[3] for r in recs)
        nbytes = sum(r[4] for r in recs)
        return {"launches": n, "avg_us": 1e3 * tot_ms / max(n, 1), "flops_per_launch": flops / max(n, 1),
                "bytes_per_launch": nbytes / max(n, 1), "tflops": flops / (tot_ms * 1e-3) / 1e12 if n else 0.0,
                "gbs": nbytes / (tot_ms * 1e-3) / 1e9 if n else 0.0}


_PROBE: Optional[KernelProbe] = None
_TAG = ""  # the tower a probed GEMM belongs to ("vision" / "text"), set by the engine around each tower


def set_probe(probe: Optional[KernelProbe]):
    global _PROBE
    _PROBE = probe


class probe_tag:
    """with ops.probe_tag("text"): GEMM probe records are keyed "gemm/text"."""

    def __init__(self, tag: str):
        self.tag = tag

    def __enter__(self):
        global _TAG
        self.prev, _TAG = _TAG, self.tag

    def __exit__(self, *a):
        global _TAG
        _TAG = self.prev


def _gkey():
    return f"gemm/{_TAG}" if _TAG else "gemm"


def _p(t: Optional[torch.Tensor]):
    return ctypes.c_void_p(t.data_ptr()) if t is not None else None


def _s():
    return ctypes.c_void_p(torch.cuda.current_stream().cuda_stream)


def _ld(t: torch.Tensor) -> int:
    assert t.dim() == 2 and t.stride(1) == 1, "row-major 2-D view required"
    return t.stride(0)


def _gemm_bytes(M, N, K, C, aux=None, a_bytes=2, b_bytes=2) -> float:
    """Algorithmic bytes of one GEMM launch: A and B read once, C written once (at its element size), and
    the epilogue's aux operand (residual read, pre-activation written or read: M x N fp16) once."""
    return a_bytes * M * K + b_bytes * N * K + C.element_size() * M * N + (2.0 * M * N if aux is not None else 0.0)


def _hbm(key: str, nbytes: float):
    """HIP-event probe around a streaming (HBM-bound) kernel: algorithmic bytes per launch."""
    if _PROBE is not None and _PROBE.wants("hbm"):
        return _PROBE.around(0.0, nbytes, key)
    return None


def _rec(ev):
    if ev is not None:
        ev.record()


def gemm_nt(A, B, C=None, bias=None, aux_in=None, aux_out=None, epilogue=EPI_NONE, tile=0):
    """C[M,N] = epi(A[M,K] . B[N,K]^T)."""
    M, K = A.shape
    N, K2 = B.shape
    assert K == K2, (A.shape, B.shape)
    if C is None:
        C = torch.empty(M, N, device=A.device, dtype=torch.float32 if epilogue == EPI_F32 else torch.float16)
    aux = aux_in if aux_in is not None else aux_out
    ld_aux = _ld(aux) if aux is not None else 0
    ev = None
    if _PROBE is not None and _PROBE.wants("gemm"):
        ev = _PROBE.around(2.0 * M * N * K, _gemm_bytes(M, N, K, C, aux), _gkey(), (M, N, K, epilogue))
    call("mf_gemm_nt", _p(A), _ld(A), _p(B), _ld(B), _p(C), _ld(C), M, N, K, _p(bias), _p(aux_in), _p(aux_out),
         ld_aux, epilogue, tile, _s())
    if ev is not None:
        ev.record()
    return C


def gemm(A, B, C=None, bias=None, aux_in=None, aux_out=None, epilogue=EPI_NONE, tile=0, a_kmajor=False,
         b_kmajor=False):
    """C[M,N] = epi(op(A) . op(B)^T): A is [M,K] (or [K,M] when a_kmajor), B is [N,K] (or [K,N]
    when b_kmajor) -- the K-major forms read dY^T / X / W of the backward products in place."""
    M, Ka = (A.shape[1], A.shape[0]) if a_kmajor else A.shape
    N, Kb = (B.shape[1], B.shape[0]) if b_kmajor else B.shape
    assert Ka == Kb, (A.shape, a_kmajor, B.shape, b_kmajor)
    K = Ka
    if C is None:
        C = torch.empty(M, N, device=A.device, dtype=torch.float32 if epilogue == EPI_F32 else torch.float16)
    aux = aux_in if aux_in is not None else aux_out
    ld_aux = _ld(aux) if aux is not None else 0
    ev = None
    if _PROBE is not None and _PROBE.wants("gemm"):
        ev = _PROBE.around(2.0 * M * N * K, _gemm_bytes(M, N, K, C, aux), _gkey(), (M, N, K, epilogue))
    call("mf_gemm", _p(A), _ld(A), int(a_kmajor), _p(B), _ld(B), int(b_kmajor), _p(C), _ld(C), M, N, K, _p(bias),
         _p(aux_in), _p(aux_out), ld_aux, epilogue, tile, _s())
    if ev is not None:
        ev.record()
    return C



def gemm_splitk_ws_floats(M: int, N: int, K: int, splits: int = 0) -> int:
    n = call("mf_gemm_splitk_ws_floats", M, N, K, splits)
    if n < 0:
        raise ValueError("split-K workspace exceeds 2^31 floats")
    return n


def gemm_splitk(A, B, C, ws, splits=0, a_kmajor=False, b_kmajor=False):
    """C[M,N] = op(A) . op(B)^T with K split over workgroups and an fp32 workspace (mf_gemm_splitk):
    for the weight gradients, few output tiles and K = tokens.  C fp16 or fp32."""
    M, Ka = (A.shape[1], A.shape[0]) if a_kmajor else A.shape
    N, Kb = (B.shape[1], B.shape[0]) if b_kmajor else B.shape
    assert Ka == Kb, (A.shape, a_kmajor, B.shape, b_kmajor)
    K = Ka
    assert ws.dtype == torch.float32 and C.dtype in (torch.float16, torch.float32)
    ev = None
    if _PROBE is not None and _PROBE.wants("gemm"):
        ev = _PROBE.around(2.0 * M * N * K, _gemm_bytes(M, N, K, C), _gkey(), (M, N, K, "splitk"))
    call("mf_gemm_splitk", _p(A), _ld(A), int(a_kmajor), _p(B), _ld(B), int(b_kmajor), _p(C), _ld(C), M, N, K,
         _p(ws), ws.numel(), splits, int(C.dtype == torch.float16), _s())
    if ev is not None:
        ev.record()
    return C


def layernorm_fwd(x, gamma, beta, y=None, mean=None, rstd=None, row_index=None):
    rows = row_index.numel() if row_index is not None else x.shape[0]
    D = x.shape[1]
    if y is None:
        y = torch.empty(rows, D, device=x.device, dtype=torch.float16)
    if mean is None:
        mean = torch.empty(rows, device=x.device, dtype=torch.float32)
    if rstd is None:
        rstd = torch.empty(rows, device=x.device, dtype=torch.float32)
    # x read, y written (fp16), mean / rstd written (fp32)
    ev = _hbm(f"layernorm_fwd/D{D}", rows * D * 4.0 + rows * 8.0)
    call("mf_layernorm_fwd", _p(x), _ld(x), _p(row_index), _p(gamma), _p(beta), _p(y), _ld(y), _p(mean), _p(rstd),
         rows, D, _s())
    _rec(ev)
    return y, mean, rstd




def layernorm_fwd_inject(x, gamma, beta, y, mean, rstd, prompt, L, row0, nrows):
    """prompt_inject_fwd(x, prompt, ...) + layernorm_fwd(x, ...) in one kernel (bit-identical)."""
    rows, D = x.shape
    ev = _hbm(f"layernorm_fwd/D{D}", rows * D * 4.0 + rows * 8.0)
    call("mf_layernorm_fwd_inject", _p(x), _ld(x), _p(gamma), _p(beta), _p(y), _ld(y), _p(mean), _p(rstd), rows, D,
         _p(prompt), L, row0, nrows, _s())
    _rec(ev)
    return y, mean, rstd


def layernorm_ws_floats(rows: int, D: int) -> int:
    return 2 * call("mf_layernorm_bwd_blocks", rows) * D


def layernorm_bwd(dy, x, gamma, mean, rstd, dx, dgamma, dbeta, workspace=None, dres=None, row_index=None,
                  accumulate=False):
    rows, D = dy.shape
    if workspace is None:
        workspace = torch.empty(layernorm_ws_floats(rows, D), device=dy.device, dtype=torch.float32)
    call("mf_layernorm_bwd", _p(dy), _ld(dy), _p(x), _ld(x), _p(row_index), _p(gamma), _p(mean), _p(rstd), _p(dres),
         _ld(dres) if dres is not None else 0, _p(dx), _ld(dx), _p(dgamma), _p(dbeta), _p(workspace), rows, D,
         int(accumulate), _s())
    return dx


class LNGradBatch:
    """Deferred dgamma/dbeta reductions of every LayerNorm backward of a pass: each LN param pair gets
    its own partial-sum workspace, and one mf_col_reduce_batch launch at the end of the backward
    reduces them all (instead of one reduction launch per LayerNorm)."""

    def __init__(self, device):
        self.device = device
        self.ws = {}          # dgamma data_ptr -> workspace
        self.descs = []       # (part_ptr, out_ptr, nblk, C)
        self.keys = []
        self.dev_descs = None
        self.max_cols = 0

    def bwd(self, dy, x, gamma, mean, rstd, dx, dgamma, dbeta, dres=None, row_index=None, live=None):
        """live = (L_live, L_full): dy / x / dx are the first L_live rows of each L_full-row sequence of a tower
        whose other rows have zero gradient (mf_layernorm_bwd_live: the full tower's partials)."""
        if live is not None:
            return self._bwd_live(dy, x, gamma, mean, rstd, dx, dgamma, dbeta, dres, live, None, 0, 0)
        rows, D = dy.shape
        key = dgamma.data_ptr()
        if key not in self.ws:
            nblk = call("mf_layernorm_bwd_blocks", rows)
            w = torch.empty(2 * nblk * D, device=self.device, dtype=torch.float32)
            self.ws[key] = w
            self.descs.append((w.data_ptr(), dgamma.data_ptr(), nblk, D))
            self.descs.append((w.data_ptr() + 4 * nblk * D, dbeta.data_ptr(), nblk, D))
            self.max_cols = max(self.max_cols, D)
            self.dev_descs = None
        # dy, x (and the residual gradient) read, dx written (fp16); mean / rstd read; dgamma / dbeta partials
        ev = _hbm(f"layernorm_bwd/D{D}", rows * D * (6.0 + (2.0 if dres is not None else 0.0)) + rows * 8.0
                  + self.ws[key].numel() * 4.0)
        call("mf_layernorm_bwd", _p(dy), _ld(dy), _p(x), _ld(x), _p(row_index), _p(gamma), _p(mean), _p(rstd),
             _p(dres), _ld(dres) if dres is not None else 0, _p(dx), _ld(dx), None, None, _p(self.ws[key]), rows, D,
             0, _s())
        _rec(ev)
        return dx

    def _ws_for(self, dgamma, dbeta, rows, D):
        key = dgamma.data_ptr()
        if key not in self.ws:
            nblk = call("mf_layernorm_bwd_blocks", rows)
            w = torch.empty(2 * nblk * D, device=self.device, dtype=torch.float32)
            self.ws[key] = w
            self.descs.append((w.data_ptr(), dgamma.data_ptr(), nblk, D))
            self.descs.append((w.data_ptr() + 4 * nblk * D, dbeta.data_ptr(), nblk, D))
            self.max_cols = max(self.max_cols, D)
            self.dev_descs = None
        return self.ws[key]

    def _inj_ws_for(self, prompt_grad, n, nrows, D):
        ikey = ("inj", prompt_grad.data_ptr())
        if ikey not in self.ws:
            part = torch.empty(n * nrows * D, device=self.device, dtype=torch.float32)
            self.ws[ikey] = part
            self.descs.append((part.data_ptr(), prompt_grad.data_ptr(), n, nrows * D))
            self.max_cols = max(self.max_cols, nrows * D)
            self.dev_descs = None
        return self.ws[ikey]

    def _bwd_live(self, dy, x, gamma, mean, rstd, dx, dgamma, dbeta, dres, live, prompt_grad, row0, nrows):
        L_live, L_full = live
        rows, D = dy.shape
        assert rows % L_live == 0 and L_live <= L_full
        seqs = rows // L_live
        ws = self._ws_for(dgamma, dbeta, seqs * L_full, D)
        inj = None
        if prompt_grad is not None:
            assert prompt_grad.dtype == torch.float32 and prompt_grad.is_contiguous()
            inj = self._inj_ws_for(prompt_grad, seqs, nrows, D)
        ev = _hbm(f"layernorm_bwd/D{D}", rows * D * (6.0 + (2.0 if dres is not None else 0.0)) + rows * 8.0
                  + (ws.numel() + (inj.numel() if inj is not None else 0)) * 4.0)
        call("mf_layernorm_bwd_live", _p(dy), _ld(dy), _p(x), _ld(x), _p(gamma), _p(mean), _p(rstd), _p(dres),
             _ld(dres) if dres is not None else 0, _p(dx), _ld(dx), _p(ws), seqs, L_live, L_full, D, _p(inj), row0,
             nrows, _s())
        _rec(ev)
        return dx

    def bwd_inject(self, dy, x, gamma, mean, rstd, dx, dgamma, dbeta, dres, prompt_grad, L, row0, nrows, live=None):
        """bwd() with the deep-prompt injection backward of the same rows fused in
        (mf_layernorm_bwd_inject): prompt_grad (fp32 [nrows, D]) = sum over sequences of those rows' dx,
        reduced in finish() with the LayerNorm partials; the rows of dx are zeroed.  live: see bwd() (then
        L must be its L_live)."""
        if live is not None:
            assert L == live[0]
            return self._bwd_live(dy, x, gamma, mean, rstd, dx, dgamma, dbeta, dres, live, prompt_grad, row0, nrows)
        rows, D = dy.shape
        assert prompt_grad.dtype == torch.float32 and prompt_grad.is_contiguous() and prompt_grad.numel() == nrows * D
        key = dgamma.data_ptr()
        if key not in self.ws:
            nblk = call("mf_layernorm_bwd_blocks", rows)
            w = torch.empty(2 * nblk * D, device=self.device, dtype=torch.float32)
            self.ws[key] = w
            self.descs.append((w.data_ptr(), dgamma.data_ptr(), nblk, D))
            self.descs.append((w.data_ptr() + 4 * nblk * D, dbeta.data_ptr(), nblk, D))
            self.max_cols = max(self.max_cols, D)
            self.dev_descs = None
        ikey = ("inj", prompt_grad.data_ptr())
        if ikey not in self.ws:
            n = rows // L
            part = torch.empty(n * nrows * D, device=self.device, dtype=torch.float32)
            self.ws[ikey] = part
            self.descs.append((part.data_ptr(), prompt_grad.data_ptr(), n, nrows * D))
            self.max_cols = max(self.max_cols, nrows * D)
            self.dev_descs = None
        ev = _hbm(f"layernorm_bwd/D{D}", rows * D * (6.0 + (2.0 if dres is not None else 0.0)) + rows * 8.0
                  + (self.ws[key].numel() + self.ws[ikey].numel()) * 4.0)
        call("mf_layernorm_bwd_inject", _p(dy), _ld(dy), _p(x), _ld(x), _p(gamma), _p(mean), _p(rstd), _p(dres),
             _ld(dres) if dres is not None else 0, _p(dx), _ld(dx), _p(self.ws[key]), rows, D, _p(self.ws[ikey]), L,
             row0, nrows, _s())
        _rec(ev)
        return dx

    def finish(self):
        if not self.descs:
            return
        if self.dev_descs is None:
            import numpy as np
            assert call("mf_col_reduce_desc_bytes") == 32
            arr = np.zeros(len(self.descs), dtype=np.dtype([("part", np.uint64), ("out", np.uint64),
                                                            ("nblk", np.int32), ("C", np.int32),
                                                            ("acc", np.int32), ("pad", np.int32)]))
            for i, (pp, op, nb, c) in enumerate(self.descs):
                arr[i] = (pp, op, nb, c, 0, 0)
            self.dev_descs = torch.from_numpy(arr.view(np.uint8)).to(self.device)
        call("mf_col_reduce_batch", _p(self.dev_descs), len(self.descs), self.max_cols, _s())


def attention_fwd(qkv, N, L, H, causal, out=None, lse=None, ld_lse=None):
    D = H * 64
    if out is None:
        out = torch.empty(N * L, D, device=qkv.device, dtype=torch.float16)
    if ld_lse is None:
        ld_lse = L
    if lse is None:
        lse = torch.empty(N * H * ld_lse, device=qkv.device, dtype=torch.float32)
    ev = None
    if _PROBE is not None and _PROBE.wants("attention"):
        # algorithmic: QK^T + PV = 4 * pairs * 64 flop per (sequence, head), pairs = L^2 (L(L+1)/2 under
        # the causal mask); bytes: Q, K, V read + O written (fp16) + the LSE (fp32)
        pairs = L * (L + 1) / 2 if causal else L * L
        ev = _PROBE.around(4.0 * N * H * pairs * 64, N * H * L * (2.0 * 4 * 64 + 4), f"attention_fwd/L{L}")
    call("mf_attention_fwd", _p(qkv), _ld(qkv), _p(out), _ld(out), _p(lse), ld_lse, N, L, H, int(causal), _s())
    if ev is not None:
        ev.record()
    return out, lse


def attention_fwd_rows(qkv, N, L, H, causal, q_rows, out, lse, ld_lse=None):
    """attention_fwd for query rows 0 .. q_rows-1 of every head only (their 16-row tiles are computed and stored;
    each row bit-identical to attention_fwd's): out / lse rows of the other queries are left untouched."""
    if ld_lse is None:
        ld_lse = L
    ev = None
    if _PROBE is not None and _PROBE.wants("attention"):
        rows = min(L, (q_rows + 15) // 16 * 16)
        ev = _PROBE.around(4.0 * N * H * rows * L * 64, N * H * (2.0 * 2 * 64 * L + 2.0 * 2 * 64 * rows),
                           f"attention_fwd_rows/L{L}")
    call("mf_attention_fwd_rows", _p(qkv), _ld(qkv), _p(out), _ld(out), _p(lse), ld_lse, N, L, H, int(causal), q_rows,
         _s())
    if ev is not None:
        ev.record()
    return out, lse


def qkv_attention_supported(N, L, H, causal) -> bool:
    return bool(call("mf_qkv_attention_supported", N, L, H, int(causal)))


def qkv_attention_fwd(x, w, bias, qkv, out, lse, N, L, H, causal, ld_lse=None):
    """The in-projection (qkv = x w^T + bias, fp16) and the attention forward in one launch
    (mf_qkv_attention_fwd): qkv [N*L, 3D] is written too (the backward reads it)."""
    D = H * 64
    if ld_lse is None:
        ld_lse = L
    assert x.shape[1] == D and tuple(w.shape) == (3 * D, D) and bias.numel() == 3 * D
    ev = None
    if _PROBE is not None and _PROBE.wants("attention"):
        # algorithmic: the in-projection 2 * (N*L) * 3D * D plus QK^T + PV; bytes: x and W read, qkv, O (fp16)
        # and the LSE written -- the round trip of qkv between two launches is gone
        pairs = L * (L + 1) / 2 if causal else L * L
        flops = 2.0 * N * L * 3 * D * D + 4.0 * N * H * pairs * 64
        nbytes = 2.0 * N * L * D + 2.0 * 3 * D * D + 2.0 * N * L * 3 * D + 2.0 * N * L * D + 4.0 * N * H * L
        ev = _PROBE.around(flops, nbytes, f"attention_fused_fwd/L{L}")
    call("mf_qkv_attention_fwd", _p(x), _ld(x), x.shape[0], _p(w), _p(bias), _p(qkv), _ld(qkv), _p(out), _ld(out),
         _p(lse), ld_lse, N, L, H, int(causal), _s())
    if ev is not None:
        ev.record()
    return out, lse


def attention_bwd(qkv, out, dout, lse, N, L, H, causal, dqkv=None, ws=None, ld_lse=None):
    if ld_lse is None:
        ld_lse = L
    if dqkv is None:
        dqkv = torch.empty_like(qkv)
    if ws is None:
        ws = torch.empty(N * H * ld_lse, device=qkv.device, dtype=torch.float32)
    ev = None
    if _PROBE is not None and _PROBE.wants("attention"):
        # algorithmic: dV = P^T dO, dP = dO V^T, dK = dS^T Q, dQ = dS K: 8 * pairs * 64 flop (the
        # recompute of S is not counted); bytes: Q, K, V, O, dO + LSE read, dQ, dK, dV written
        pairs = L * (L + 1) / 2 if causal else L * L
        ev = _PROBE.around(8.0 * N * H * pairs * 64, N * H * L * (2.0 * 8 * 64 + 4), f"attention_bwd/L{L}")
    call("mf_attention_bwd", _p(qkv), _ld(qkv), _p(out), _ld(out), _p(dout), _ld(dout), _p(lse), _p(ws), ld_lse,
         _p(dqkv), _ld(dqkv), N, L, H, int(causal), _s())
    if ev is not None:
        ev.record()
    return dqkv


def im2col_patch(img, out, patch=16):
    B, C, R, R2 = img.shape
    assert C == 3 and R == R2 and img.is_contiguous()
    call("mf_im2col_patch", _p(img), int(img.dtype == torch.float32), _p(out), B, R, patch, _s())
    return out


def vision_assemble(patch, cls, pos, shared_ctx, x, B, G2, n_ctx, D):
    call("mf_vision_assemble", _p(patch), _p(cls), _p(pos), _p(shared_ctx), _p(x), B, G2, n_ctx, D, _s())
    return x


def text_assemble(prefix, ctx, suffix, pos, x, K, L, n_ctx, D):
    call("mf_text_assemble", _p(prefix), _p(ctx), _p(suffix), _p(pos), _p(x), K, L, n_ctx, D, _s())
    return x


def prompt_inject_fwd(x, prompt, N, L, row0, nrows, D):
    call("mf_prompt_inject_fwd", _p(x), _p(prompt), N, L, row0, nrows, D, _s())


def prompt_inject_bwd(dx, N, L, row0, nrows, D, out, accumulate=False, zero_rows=True):
    call("mf_prompt_inject_bwd", _p(dx), N, L, row0, nrows, D, _p(out), int(out.dtype == torch.float16),
         int(accumulate), int(zero_rows), _s())


def seq_grow(src, dst, cap, prompt, N, Lp, ncap, n_ctx, D):
    """dst [N*(Lp+ncap), D] = per sequence: src rows [0, Lp-n_ctx) | cap [ncap, D] | fp16(prompt [n_ctx, D])."""
    assert src.shape[0] == N * Lp and dst.shape[0] == N * (Lp + ncap) and prompt.dtype == torch.float32
    call("mf_seq_grow", _p(src), _p(dst), _p(cap), _p(prompt), N, Lp, ncap, n_ctx, D, _s())


def seq_scatter(src, dst, N, L_live, L_full):
    """dst rows n*L_full + t = src rows n*L_live + t (t < L_live), src's columns; dst's other rows untouched."""
    C = src.shape[1]
    assert src.shape[0] == N * L_live and dst.shape[0] >= N * L_full and dst.shape[1] >= C
    ev = _hbm("seq_scatter", 4.0 * N * L_live * C)
    call("mf_seq_scatter", _p(src), _ld(src), _p(dst), _ld(dst), N, L_live, L_full, C, _s())
    _rec(ev)
    return dst


def seq_grow_bwd(ddst, dsrc, N, Lp, ncap, n_ctx, D):
    assert ddst.shape[0] == N * (Lp + ncap) and dsrc.shape[0] == N * Lp
    call("mf_seq_grow_bwd", _p(ddst), _p(dsrc), N, Lp, ncap, n_ctx, D, _s())


def caption_pool(tokens, table, w, pooled):
    """tokens int32 [B, T] on the device, table fp32 [vocab, D], w fp16 [D] -> pooled fp16 [B, D]."""
    B, T = tokens.shape
    assert tokens.dtype == torch.int32 and table.dtype == torch.float32 and w.dtype == torch.float16
    call("mf_caption_pool", _p(tokens), B, T, _p(table), table.shape[0], _p(w), table.shape[1], _p(pooled), _s())
    return pooled


def transpose(inp, out):
    R, C = inp.shape
    call("mf_transpose_f16", _p(inp), _ld(inp), _p(out), _ld(out), R, C, _s())
    return out


def colsum_ws_floats(R: int, C: int) -> int:
    return call("mf_colsum_blocks", R) * C


def colsum(inp, out, workspace=None):
    R, C = inp.shape
    if workspace is None:
        workspace = torch.empty(colsum_ws_floats(R, C), device=inp.device, dtype=torch.float32)
    call("mf_colsum_f16", _p(inp), _ld(inp), R, C, _p(out), int(out.dtype == torch.float16), _p(workspace), _s())
    return out


def small_linear_fwd(X, W, b, Y):
    M, I = X.shape
    O = W.shape[0]
    call("mf_small_linear_fwd", _p(X), _p(W), _p(b), _p(Y), M, I, O, int(X.dtype == torch.float16), _s())
    return Y


class SmallLinearBatch:
    """A fixed set of small Linears (the prompt learner's) run as one launch per direction.  Each entry:
    X [M,I], W [O,I], b [O] or None, Y [M,O]; backward: dY [M,O], dX (accumulated when acc_dx), dW, db.
    The descriptor table is built once (static pointers, hipGraph-capturable)."""

    def __init__(self, device, entries):
        import numpy as np
        assert call("mf_small_linear_desc_bytes") == 88
        dt = np.dtype([("X", np.uint64), ("W", np.uint64), ("b", np.uint64), ("Y", np.uint64), ("dY", np.uint64),
                       ("dX", np.uint64), ("dW", np.uint64), ("db", np.uint64), ("M", np.int32), ("I", np.int32),
                       ("O", np.int32), ("is16", np.int32), ("acc", np.int32), ("pad", np.int32)])
        arr = np.zeros(len(entries), dtype=dt)
        ptr = lambda t: 0 if t is None else t.data_ptr()
        self.max_mo = self.max_m = self.max_i = self.max_oi = 0
        for k, e in enumerate(entries):
            M, I = e["X"].shape
            O = e["W"].shape[0]
            arr[k] = (ptr(e["X"]), ptr(e["W"]), ptr(e.get("b")), ptr(e["Y"]), ptr(e.get("dY")), ptr(e.get("dX")),
                      ptr(e.get("dW")), ptr(e.get("db")), M, I, O, int(e["X"].dtype == torch.float16),
                      int(e.get("acc_dx", False)), 0)
            self.max_mo, self.max_m = max(self.max_mo, M * O), max(self.max_m, M)
            self.max_i, self.max_oi = max(self.max_i, I), max(self.max_oi, O * I)
        self.n = len(entries)
        self.descs = torch.from_numpy(arr.view(np.uint8)).to(device)

    def fwd(self):
        call("mf_small_linear_fwd_batch", _p(self.descs), self.n, self.max_mo, _s())

    def bwd(self):
        call("mf_small_linear_bwd_batch", _p(self.descs), self.n, self.max_m, self.max_i, self.max_oi, _s())


def small_linear_bwd(dY, X, W, dX=None, dW=None, db=None, accumulate_dx=False):
    M, I = X.shape
    O = W.shape[0]
    call("mf_small_linear_bwd", _p(dY), _p(X), _p(W), _p(dX), _p(dW), _p(db), M, I, O,
         int(X.dtype == torch.float16), int(accumulate_dx), _s())


def clip_head_fwd(img, txt, logit_scale, img_n, txt_n, norms, mm, logits):
    B, D = img.shape
    K = txt.shape[0]
    call("mf_clip_head_fwd", _p(img), _p(txt), B, K, D, _p(logit_scale), _p(img_n), _p(txt_n), _p(norms), _p(mm),
         _p(logits), _s())


def clip_loss_fwd_bwd(img, txt, img_n, txt_n, norms, logits, label, logit_scale, dmm, cos_ws, loss_out, dimg_n,
                      dtxt_n, dimg, dtxt):
    B, D = img.shape
    K = txt.shape[0]
    call("mf_clip_loss_fwd_bwd", _p(img), _p(txt), _p(img_n), _p(txt_n), _p(norms), _p(logits), _p(label), B, K, D,
         _p(logit_scale), _p(dmm), _p(cos_ws), _p(loss_out), _p(dimg_n), _p(dtxt_n), _p(dimg), _p(dtxt), _s())



def clip_loss_soft_fwd_bwd(img, txt, img_n, txt_n, norms, logits, label_probs, logit_scale, dmm, cos_ws, soft_ws,
                           loss_out, dimg_n, dtxt_n, dimg, dtxt):
    """Soft-label branch (trainers/maple.py:356-360): label_probs fp32 [B, K]; soft_ws fp16 >= 2*B*D."""
    B, D = img.shape
    K = txt.shape[0]
    if label_probs.dtype != torch.float32 or tuple(label_probs.shape) != (B, K) or not label_probs.is_contiguous():
        raise ValueError(f"soft labels must be contiguous fp32 [{B}, {K}], got {label_probs.dtype} "
                         f"{tuple(label_probs.shape)}")
    if soft_ws.dtype != torch.float16 or soft_ws.numel() < 2 * B * D:
        raise ValueError("soft_ws: fp16 workspace of 2*B*D elements")
    call("mf_clip_loss_soft_fwd_bwd", _p(img), _p(txt), _p(img_n), _p(txt_n), _p(norms), _p(logits),
         _p(label_probs), B, K, D, _p(logit_scale), _p(dmm), _p(cos_ws), _p(soft_ws), _p(loss_out), _p(dimg_n),
         _p(dtxt_n), _p(dimg), _p(dtxt), _s())


def argmax_correct(logits, label=None, pred=None, acc=None):
    B, K = logits.shape
    call("mf_argmax_correct", _p(logits), B, K, _p(label), _p(pred), _p(acc), _s())


def optim_chunk_elems() -> int:
    return call("mf_optim_chunk_elems")


def clip_grad_norm(g16, g32, chunks, nchunks, max_norm, part, out):
    ev = _hbm("clip_grad_norm", g16.numel() * 2.0 + g32.numel() * 4.0)  # every gradient read once
    call("mf_clip_grad_norm", _p(g16), _p(g32), _p(chunks), nchunks, float(max_norm), _p(part), _p(out), _s())
    _rec(ev)


def sgd_step(p, g, buf, coef, hyper):
    """hyper: device fp32 tensor {lr, momentum, weight_decay, first_step}."""
    # p, g, momentum read; p, momentum written (each at the parameter's element size)
    ev = _hbm(f"sgd_step/{'f16' if p.dtype == torch.float16 else 'f32'}", p.numel() * 5.0 * p.element_size())
    call("mf_sgd_step", _p(p), _p(g), _p(buf), p.numel(), int(p.dtype == torch.float16), _p(coef), _p(hyper), _s())
    _rec(ev)


def optimizer_step(p16, g16, b16, p32, g32, b32, chunks, nchunks, max_norm, part, out, hyper, halt_src,
                   input_flag=None):
    """clip_grad_norm + sgd_step(fp16) + sgd_step(fp32), with hyper[4] = max(hyper[4], halt_src[0], input_flag[0])
    folded in: three launches, bit-identical (mf_optimizer_step)."""
    nb = g16.numel() * 2.0 + g32.numel() * 4.0 + p16.numel() * 10.0 + p32.numel() * 20.0
    ev = _hbm("optimizer_step", nb)  # every gradient read twice; p, g, momentum read and written
    call("mf_optimizer_step", _p(p16), _p(g16), _p(b16), p16.numel(), _p(p32), _p(g32), _p(b32), p32.numel(), _p(chunks),
         nchunks, float(max_norm), _p(part), _p(out), _p(hyper), _p(halt_src), _p(input_flag), _s())
    _rec(ev)


def fedavg_pack(p16, p32, invalid_flag, bucket):
    """bucket: n16 + n32 + 1 floats (last = this client's valid vote)."""
    assert bucket.numel() == p16.numel() + p32.numel() + 1
    call("mf_fedavg_pack", _p(p16), p16.numel(), _p(p32), p32.numel(), _p(invalid_flag), _p(bucket), _s())


def fedavg_unpack(bucket, p16, p32, g16=None, g32=None):
    call("mf_fedavg_unpack", _p(bucket), _p(p16), p16.numel(), _p(p32), p32.numel(), _p(g16), _p(g32), _s())


def fedavg_reduce_ordered(gathered, nclients, out):
    """out = sum over clients (in client order) of gathered.view(nclients, -1)[:, :out.numel()]."""
    stride = gathered.numel() // nclients
    assert gathered.numel() == stride * nclients and out.numel() <= stride
    call("mf_fedavg_reduce_ordered", _p(gathered), nclients, stride, out.numel(), _p(out), _s())


def nonfinite_flag(x, flag):
    call("mf_nonfinite_flag", _p(x), x.numel(), int(x.dtype == torch.float16), _p(flag), _s())
