"""Horizon sharding across GPUs (one process per GPU), DESIGN.md section 6.

Rank r owns stages [N0_r, N1_r) of one long horizon (config C4: N = 65536,
nx = 24, nu = 8 over 8 x MI355X).  Each rank
  1. solves its slice as a PARALLEL handle (segments + local scans) and exports
     its slice element e_r = (F, C, f, P, p)           -> pdplqr_shard_backward
  2. all-gathers the R elements (3n^2 + 2n doubles each) over RCCL/xGMI
  3. folds the global prefix (ranks < r) and suffix (ranks > r), computes the
     boundary states of its segments and rolls out      -> pdplqr_shard_forward
backward_without_factorization (an ADMM iteration with rho unchanged,
lqr_solver_parallel.hpp:148-154,190-211) reuses every factorization: only the
elements' (f, p) change, so step 2 exchanges 2n doubles per problem instead of
3n^2 + 2n and the rest of the last full gather is kept   -> solve_distributed(..., factorize=False)
This is the multi-GPU form of the reference's condensed segment system
(condensed_system.hpp:8-299), whose serial fold over OpenMP segments is
replaced by the associative combine.
"""
from __future__ import annotations

import ctypes as C
from typing import List, Tuple

import numpy as np

from . import _lib
from ._lib import check, lib
from .solvers import _Handle, _mem_of, _ptr


def split_horizon(N: int, R: int) -> List[Tuple[int, int]]:
    """Contiguous, balanced slices [N0, N1) of the horizon, one per rank."""
    base, extra = divmod(N, R)
    out, st = [], 0
    for r in range(R):
        ln = base + (1 if r < extra else 0)
        out.append((st, st + ln))
        st += ln
    return out


def slice_arrays(E, c, H, h, n, m, N, N0, N1, last):
    """Local boundary arrays of the slice [N0, N1) from batch-major full arrays.
    Non-final slices get a zero terminal block (unused: their last segment uses
    the dummy zero terminal, lqr_kernel_parallel.hpp:60-66)."""
    s = n + m
    xp = _xp(E)
    B = E.shape[0]
    El = E[:, N0 * n * s:N1 * n * s]
    cl = c[:, N0 * n:N1 * n]
    Hs = H[:, N0 * s * s:N1 * s * s]
    hs = h[:, N0 * s:N1 * s]
    if last:
        HN, hN = H[:, N * s * s:], h[:, N * s:]
    else:
        HN = xp.zeros((B, n * n), dtype=H.dtype, **_dev(H))
        hN = xp.zeros((B, n), dtype=h.dtype, **_dev(h))
    cat = xp.concatenate if xp is np else xp.cat
    return (_contig(El), _contig(cl), _contig(cat([Hs, HN], 1)), _contig(cat([hs, hN], 1)))


def _xp(a):
    if isinstance(a, np.ndarray):
        return np
    import torch

    return torch


def _dev(a):
    return {} if isinstance(a, np.ndarray) else {"device": a.device}


def _contig(a):
    return np.ascontiguousarray(a) if isinstance(a, np.ndarray) else a.contiguous()


class HorizonShard:
    """One rank's slice of a horizon-sharded solve (batch problems share the split)."""

    def __init__(self, n: int, m: int, N_local: int, batch: int = 1, device: int = 0, segment_len: int = 0,
                 ncs=None, condensed: str = "CHOLESKY"):
        """``condensed`` picks the form of every segment / rank combine, as
        ``CondensedSystemSolverType`` does for ``LQRParallelSolver``
        (lqr_solver_parallel.hpp:14-17): CHOLESKY (default; needs positive
        definite value functions at the boundaries) or LU (semidefinite ones
        too).  The device segmentation is internal (segment_len); the handle's
        reference segment count only has to satisfy CHOLESKY's ns >= 2."""
        self.n, self.m, self.N, self.batch = n, m, N_local, batch
        self.es = 3 * n * n + 2 * n
        ctype = {"LU": _lib.PDPLQR_CONDENSED_LU, "CHOLESKY": _lib.PDPLQR_CONDENSED_CHOLESKY}[condensed]
        ns = 2 if ctype == _lib.PDPLQR_CONDENSED_CHOLESKY and N_local >= 3 else 1
        if ns == 1:
            ctype = _lib.PDPLQR_CONDENSED_LU  # a slice of < 3 stages: one reference segment
        self.condensed = "CHOLESKY" if ctype == _lib.PDPLQR_CONDENSED_CHOLESKY else "LU"
        self._hd = _Handle(n, m, N_local, batch, _lib.PDPLQR_SOLVER_PARALLEL, num_segments=ns,
                           condensed_type=ctype, device=device, keep_factors=True, ncs=ncs,
                           segment_len=segment_len)
        # the full all-gather of the last factorising solve_distributed and its
        # key (world size, rank, group): factorize=False writes the new (f, p)
        # into it, so anything that changes F, C, P or the ranks clears it
        self._gathered = None
        self._gather_key = None

    @property
    def handle(self):
        return self._hd

    def set_model(self, E, c, H, h, D=None):
        self._gathered = None  # the kept gather holds F, C, P of the old model
        self._hd.set_model(E, c, H, h, D)

    def update_problem_data(self, ws, ys=None, zs=None, inv_rho=None, sigma: float = 0.0):
        self._hd.update_problem_data(ws, ys, zs, inv_rho, sigma)

    def backward(self, elem_out, is_last: bool, rho=None):
        """Slice backward; writes the slice element(s) [batch, 3n^2+2n] into elem_out.
        A factorising backward outside solve_distributed invalidates the gather
        solve_distributed(factorize=False) would reuse."""
        self._gathered = None
        pr, pe = _ptr(rho, "rho"), _ptr(elem_out, "elem")
        mem = pe[1]
        check(lib().pdplqr_shard_backward(self._hd.h, pr[0], int(bool(is_last)), pe[0], mem))
        return elem_out

    def backward_without_factorization(self, elem_out, is_last: bool, rho=None):
        """Slice backward reusing the factorizations of the last backward (same
        is_last); writes the whole element, of which only f and p are new."""
        pr, pe = _ptr(rho, "rho"), _ptr(elem_out, "elem")
        check(lib().pdplqr_shard_backward_without_factorization(self._hd.h, pr[0], int(bool(is_last)), pe[0], pe[1]))
        return elem_out

    def fp_slices(self):
        """(f, p) positions inside an element (layout F C f P p, include/pdplqr.h)."""
        n = self.n
        return slice(2 * n * n, 2 * n * n + n), slice(3 * n * n + n, 3 * n * n + 2 * n)

    def forward(self, x0, elems_all, num_shards: int, shard_id: int, ws_out):
        """elems_all: [num_shards, batch, 3n^2+2n] (rank-major all-gather output)."""
        p0, pe, pw = _ptr(x0, "x0"), _ptr(elems_all, "elems"), _ptr(ws_out, "ws")
        check(lib().pdplqr_shard_forward(self._hd.h, p0[0], pe[0], int(num_shards), int(shard_id), pw[0],
                                         _mem_of(p0, pe, pw)))
        return ws_out

    def synchronize(self):
        self._hd.synchronize()

    def stream(self) -> int:
        return self._hd.stream()

    def set_stream(self, stream_ptr: int):
        """Run the shard's launches on `stream_ptr` (e.g. torch's current side
        stream: solve_distributed then needs no cross-stream joins)."""
        self._hd.set_stream(stream_ptr)

    def close(self):
        self._hd.close()


def solve_distributed(shard: HorizonShard, x0, ws_out, rho=None, group=None, factorize: bool = True):
    """backward -> all-gather of slice elements -> forward, on the current
    torch.distributed process group.  With the nccl backend (RCCL) the
    elements stay on the GPU; with gloo they are gathered through host memory.
    factorize=False: backward_without_factorization; the all-gather carries only
    every rank's (f, p) (2n doubles per problem, lqr_solver_parallel.hpp:207-210),
    written into the full gather kept from the last factorising call."""
    import torch
    import torch.distributed as dist

    world = dist.get_world_size(group)
    rank = dist.get_rank(group)
    on_gpu = dist.get_backend(group) == "nccl"
    dev = torch.device("cuda", torch.cuda.current_device()) if on_gpu else torch.device("cpu")
    last = rank == world - 1
    key = (world, rank, id(group) if group is not None else None)
    if not factorize:
        if getattr(shard, "_gathered", None) is None:
            raise RuntimeError("solve_distributed(factorize=False) needs a preceding factorising solve "
                               "(set_model / a direct backward since then invalidate it)")
        if shard._gather_key != key:
            raise RuntimeError("solve_distributed(factorize=False): the process group or world size changed "
                               "since the factorising solve")
    fs, ps = shard.fp_slices()

    def exchange(elem):
        """The all-gather: the whole elements, or their (f, p) into the kept gather."""
        if factorize:
            g = torch.empty(world, shard.batch, shard.es, dtype=torch.float64, device=elem.device)
            if on_gpu:
                dist.all_gather_into_tensor(g, elem, group=group)
            else:
                parts = [torch.empty_like(elem) for _ in range(world)]
                dist.all_gather(parts, elem, group=group)
                g = torch.stack(parts).contiguous()
            shard._gathered = g
            shard._gather_key = key
            return g
        fp = torch.cat([elem[:, fs], elem[:, ps]], dim=1).contiguous()
        gfp = torch.empty(world, shard.batch, 2 * shard.n, dtype=torch.float64, device=fp.device)
        if on_gpu:
            dist.all_gather_into_tensor(gfp, fp, group=group)
        else:
            parts = [torch.empty_like(fp) for _ in range(world)]
            dist.all_gather(parts, fp, group=group)
            gfp = torch.stack(parts)
        g = shard._gathered
        g[:, :, fs] = gfp[:, :, :shard.n]
        g[:, :, ps] = gfp[:, :, shard.n:]
        return g

    def bwd(elem):
        if factorize:
            shard.backward(elem, last, rho)
        else:
            shard.backward_without_factorization(elem, last, rho)

    elem = torch.empty(shard.batch, shard.es, dtype=torch.float64, device=dev)
    if on_gpu and shard.stream() == torch.cuda.current_stream().cuda_stream:
        # the shard runs on torch's current stream (set_stream): stream order
        # alone sequences backward, the all-gather (ProcessGroupNCCL orders its
        # stream after the current one) and forward -- no event joins, which
        # cost ~19 us of GPU timeline each (profiles/r04/c2_host.log)
        bwd(elem)
        gathered = exchange(elem)
        shard.forward(x0, gathered, world, rank, ws_out)
        return ws_out
    if on_gpu:
        # Device-side ordering between the handle's stream and torch's current
        # stream (which ProcessGroupNCCL orders the all-gather against): events,
        # no host round trip between backward, exchange and forward.
        hs = torch.cuda.ExternalStream(shard.stream(), device=dev)
        cur = torch.cuda.current_stream()
        hs.wait_stream(cur)  # x0 / ws_out / rho produced on the current stream
        elem.record_stream(hs)
        bwd(elem)
        cur.wait_stream(hs)
        gathered = exchange(elem)
        hs.wait_stream(cur)
        gathered.record_stream(hs)
        shard.forward(x0, gathered, world, rank, ws_out)
        cur.wait_stream(hs)  # ws_out is read on the current stream
        return ws_out
    e_np = np.zeros((shard.batch, shard.es))
    bwd(e_np)
    gathered = exchange(torch.from_numpy(e_np))
    if isinstance(ws_out, np.ndarray):
        gathered = gathered.numpy()
    elif getattr(ws_out, "is_cuda", False):
        gathered = gathered.to(ws_out.device)
    return shard.forward(x0, np.ascontiguousarray(gathered) if isinstance(gathered, np.ndarray) else gathered,
                         world, rank, ws_out)
