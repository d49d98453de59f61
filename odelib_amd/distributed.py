"""Walker sharding across GPUs (one process per GPU) and the posterior all-gather.

The reference's only parallelism is independent chains on a process pool
(ODElib/Framework.py:755-785, 1025-1030) followed by ``pd.concat`` of the per-chain
posteriors (Framework.py:1035-1038).  Here chains are walkers: rank r owns the
contiguous global walker ids ``[offset_r, offset_r + count_r)``, runs them with no
communication (Philox draws keyed by the GLOBAL id, so the result does not depend on
the number of GPUs), and the per-rank posterior blocks ``[kept][P+5][count_r]`` are
pooled by ONE all-gather (RCCL over xGMI with the ``nccl`` backend; gloo on CPU).
"""
from __future__ import annotations

import contextlib
import os
import sys
import threading
import time

import numpy as np


@contextlib.contextmanager
def watch(what: str, rank: int, timeout_s: float = 180.0, log: bool = True):
    """Name a collective (or a communicator set-up) in this rank's log and bound it.

    Entry and exit go to stderr as ``[rank r +t s] what: enter / exit (dt s)``, so a multi-
    rank run that stalls shows from its tail alone which rank is inside which call.  If the
    call has not returned after ``timeout_s`` the rank prints ``... did not return`` and ends
    the process with exit status 87 instead of hanging (os._exit from a watchdog thread: the
    collective cannot be interrupted; the launcher then tears the job down).  The multi-GPU
    pooling path of the reference is ``Pool.starmap`` + ``pd.concat`` (Framework.py:779-780,
    :1037); its RCCL analogue first runs with more than one rank on an 8-GPU node."""
    t0 = time.perf_counter()
    stamp = lambda: f"[rank {rank} +{time.perf_counter() - _T0:.3f} s]"  # noqa: E731
    if log:
        print(f"{stamp()} {what}: enter", file=sys.stderr, flush=True)

    def expire():
        print(f"{stamp()} {what}: did not return within {timeout_s:.0f} s — exiting (87)", file=sys.stderr,
              flush=True)
        os._exit(87)

    timer = threading.Timer(timeout_s, expire)
    timer.daemon = True
    timer.start()
    try:
        yield
    finally:
        timer.cancel()
        if log:
            print(f"{stamp()} {what}: exit ({time.perf_counter() - t0:.3f} s)", file=sys.stderr, flush=True)


_T0 = time.perf_counter()


def shard(n_total: int, rank: int, world: int) -> tuple[int, int]:
    """Contiguous balanced split: (global offset, count) of ``rank``."""
    if world < 1 or not (0 <= rank < world):
        raise ValueError("bad rank/world")
    base, extra = divmod(int(n_total), int(world))
    count = base + (1 if rank < extra else 0)
    offset = rank * base + min(rank, extra)
    return offset, count


def allgather_walkers(block, n_total: int, group=None):
    """Gather per-rank blocks [..., count_r] (walker axis last) into [..., n_total] on
    every rank, in global walker order.  Uneven shards are padded to the largest count
    for the collective and trimmed afterwards."""
    import torch
    import torch.distributed as dist
    world = dist.get_world_size(group)
    counts = [shard(n_total, r, world)[1] for r in range(world)]
    cmax = max(counts)
    lead = tuple(block.shape[:-1])
    if block.shape[-1] != counts[dist.get_rank(group)]:
        raise ValueError("block walker count does not match this rank's shard")
    padded = block
    if block.shape[-1] < cmax:
        padded = torch.zeros(lead + (cmax,), dtype=block.dtype, device=block.device)
        padded[..., :block.shape[-1]] = block
    padded = padded.contiguous()
    if dist.get_backend(group) == "nccl":
        out = torch.empty((world,) + lead + (cmax,), dtype=block.dtype, device=block.device)
        dist.all_gather_into_tensor(out, padded, group=group)
        parts = [out[r, ..., :counts[r]] for r in range(world)]
    else:
        bufs = [torch.empty_like(padded) for _ in range(world)]
        dist.all_gather(bufs, padded, group=group)
        parts = [bufs[r][..., :counts[r]] for r in range(world)]
    return torch.cat(parts, dim=-1)


def native_comm(device: int, group=None):
    """The C-ABI's RCCL communicator (``oe_comm``) over the ranks of a torch.distributed
    group: rank 0 makes the id, one broadcast hands it to the others.  Without torch a
    caller does the same with any channel."""
    import torch.distributed as dist
    from . import _native as N
    if not (dist.is_available() and dist.is_initialized()):  # one process: a 1-rank communicator
        return N.Comm(device, 1, 0, N.comm_unique_id())
    world, rank = dist.get_world_size(group), dist.get_rank(group)
    obj = [N.comm_unique_id() if rank == 0 else None]
    dist.broadcast_object_list(obj, src=dist.get_global_rank(group, 0) if group is not None else 0, group=group)
    return N.Comm(device, world, rank, obj[0])


def native_allgather_walkers(block, n_total: int, comm):
    """``allgather_walkers`` through ``oe_allgather_samples``: per-rank device blocks
    [..., count_r] (walker axis last) pooled into [..., n_total] in global walker order."""
    import torch
    counts = [shard(n_total, r, comm.n_ranks)[1] for r in range(comm.n_ranks)]
    if block.shape[-1] != counts[comm.rank]:
        raise ValueError("block walker count does not match this rank's shard")
    if block.device.type != "cuda" or block.dtype != torch.float64:
        raise ValueError("oe_allgather_samples takes float64 device tensors")
    blk = block.contiguous()
    lead = tuple(blk.shape[:-1])
    rows = int(np.prod(lead)) if lead else 1
    out = torch.empty(lead + (int(n_total),), dtype=torch.float64, device=blk.device)
    comm.set_stream(torch.cuda.current_stream(blk.device).cuda_stream)
    comm.allgather_samples(rows, blk.data_ptr(), counts, out.data_ptr())
    return out


def sharded_mh(engine, theta_all, y0_all, nits: int, burnin: int, walk_mask, init_param=None, seed: int = 0,
               step_sd: float = 0.05, group=None, speculate="auto"):
    """Run the global ensemble ``theta_all [P][W_total]`` sharded over the ranks of
    ``group`` (each rank: its shard on its own device via ``engine``), Philox draws, and
    return the pooled posterior samples [kept][P+5][W_total] (identical on all ranks).
    ``speculate``: each rank's speculative MH rounds (``Engine.mh_run``; on for shards too
    small to fill their device).  The draws are keyed by global walker id and iteration, and
    in the MH kernels every chain is integrated on its own — DOPRI5 step sizes per chain
    (csrc/lane.cuh) and, for 'auto' / 'bdf', BDF step sizes and orders per chain
    (csrc/bdf.cuh integrate_bdf_lane) — so with RK4, DOPRI5, 'auto' and 'bdf' the pooled chains are bitwise
    those of one sequential launch for any rank count and speculation depth (models of up to
    8 states; the split wide-chain kernels group 64/K chains per step size), as the
    reference's chains, one odeint call per proposal (Framework.py:656, :779-780), never
    depend on each other."""
    import torch.distributed as dist
    world, rank = dist.get_world_size(group), dist.get_rank(group)
    W = int(np.asarray(theta_all).shape[1]) if not hasattr(theta_all, "shape") else int(theta_all.shape[1])
    off, cnt = shard(W, rank, world)
    r = engine.mh_run(theta_all[:, off:off + cnt], y0_all[:, off:off + cnt], nits=nits, burnin=burnin,
                      walk_mask=walk_mask, init_param=init_param, rng="philox", seed=seed, step_sd=step_sd,
                      walker_offset=off, speculate=speculate)
    return allgather_walkers(r["samples"], W, group=group), r


def pooled_rawstats(block, n_params: int, group=None):
    """``rawstats`` (Framework.py:11-17: median = exp(mean log x), log-normal std from the
    ddof=1 std of log x) of every parameter over the POOLED posterior, from the per-rank
    sample blocks [kept][P+5][count_r] without gathering them: two all-reduces of
    per-parameter sufficient statistics (n, Σ log x, then Σ (log x − mean)²), 2P+1 and P
    doubles.  Without an initialised process group it is the single-process result.
    Returns (median [P], std [P]) as numpy arrays."""
    import torch
    import torch.distributed as dist
    dist_on = dist.is_available() and dist.is_initialized()
    P = int(n_params)
    lx = torch.log(block[:, :P, :].to(torch.float64)).permute(1, 0, 2).reshape(P, -1)  # [P][kept*count]
    dev = lx.device if (not dist_on or dist.get_backend(group) == "nccl") else torch.device("cpu")
    s1 = torch.cat([lx.sum(dim=1), torch.tensor([float(lx.shape[1])], dtype=torch.float64, device=lx.device)]).to(dev)
    if dist_on:
        dist.all_reduce(s1, group=group)
    n = s1[P]
    mean = s1[:P] / n
    s2 = ((lx - mean.to(lx.device)[:, None]) ** 2).sum(dim=1).to(dev)
    if dist_on:
        dist.all_reduce(s2, group=group)
    var = s2 / (n - 1.0)
    mean, var = mean.cpu().numpy(), var.cpu().numpy()
    median = np.exp(mean)
    std = ((np.exp(var) - 1) * np.exp(2 * mean + var)) ** 0.5
    return median, std
