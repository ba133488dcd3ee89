"""Multi-GPU sharding of streams.

Frames are independent and the per-stream state (FFTProcessor members, processSSB_opt statics) is small,
so the path shards by stream with no data-path collective: rank r owns streams [r*B, (r+1)*B) and runs its
own engine on its own GPU (weak scaling).  The one collective is the per-step gather of the 72-byte frame
records to rank 0; spectra and PCM stay on the GPU that produced them.  A consumer that
wants spectra on rank 0 gathers the focus-window slice of each frame (gather_focus: 82 bins of 16384 at
2 MHz / 5 kHz, 0.5 % of the bytes) rather than the 268 MB of full spectra per GPU per step; gather_spectra moves
the full spectra (the fftCallback payload, sdr-bridge-java-soapy.cpp:456-465) when a consumer needs them all.
"""
from __future__ import annotations


def stream_range(rank: int, world: int, streams_per_rank: int) -> tuple[int, int]:
    """[first, last) global stream ids owned by `rank`."""
    if not (0 <= rank < world) or streams_per_rank < 0:
        raise ValueError(f"bad shard rank={rank} world={world} streams_per_rank={streams_per_rank}")
    return rank * streams_per_rank, (rank + 1) * streams_per_rank


def gather_records(records, world: int, rank: int, dst: int = 0, group=None, out=None, async_op: bool = False):
    """Gather each rank's [B, record_bytes] uint8 record tensor to `dst`.

    Returns the [world*B, record_bytes] concatenation (global stream order) on `dst`, None elsewhere.  The
    tensor must live where the process group's backend expects it (HIP memory for nccl/RCCL, host for gloo).
    `out` (on dst): a preallocated [world*B, record_bytes] tensor to gather into (no per-step allocation);
    with RCCL the gather is ordered on the current stream, so no host synchronisation is needed.  With a process
    group initialised the collective runs at every world size, one rank included (so a one-GPU job drives the same
    RCCL path as an 8-GPU one); without one, world must be 1 and the tensor itself is returned.
    async_op: return (result, work) without making the current stream wait for the collective (RCCL runs it on its
    own stream after the current stream's earlier work); the caller keeps `records` (and `out`) unchanged until it
    has called work.wait() (a stream-level wait with RCCL), e.g. by rotating buffers.  work is None when no
    collective ran.
    """
    import torch
    import torch.distributed as dist

    if world == 1 and not (dist.is_available() and dist.is_initialized()):
        return (records, None) if async_op else records  # no process group: nothing to gather
    if rank == dst:
        if out is None:
            out = torch.empty((world * records.shape[0],) + tuple(records.shape[1:]), dtype=records.dtype,
                              device=records.device)
        bufs = list(out.chunk(world, dim=0))
    else:
        bufs = None
    work = dist.gather(records, bufs, dst=dst, group=group, async_op=async_op)
    res = out if rank == dst else None
    return (res, work) if async_op else res


def gather_focus(spectra, first_bin: int, n_bins: int, world: int, rank: int, dst: int = 0, group=None, out=None,
                 staging=None, async_op: bool = False):
    """Gather each rank's focus-window spectrum slice [B, n_bins] (bins [first_bin, first_bin + n_bins) of the
    [B, N] fftshifted spectra, sdrg.focus_window) to `dst` as [world*B, n_bins] float32, global stream order.

    `staging` (optional, every rank): a preallocated contiguous [B, n_bins] tensor for the slice; `out` (on dst):
    the preallocated result.  Returns the result on dst, None elsewhere (world == 1: the slice itself)."""
    import torch

    sl = spectra[:, first_bin:first_bin + n_bins]
    if staging is None:
        staging = torch.empty((spectra.shape[0], n_bins), dtype=spectra.dtype, device=spectra.device)
    staging.copy_(sl)
    return gather_records(staging, world, rank, dst=dst, group=group, out=out, async_op=async_op)


def gather_spectra(spectra, world: int, rank: int, dst: int = 0, group=None, out=None):
    """Gather each rank's full [B, N] fftshifted spectra (the fftCallback payload of every frame,
    sdr-bridge-java-soapy.cpp:456-465) to `dst` as [world*B, N] float32 in global stream order: 4*N bytes per
    frame (268 MB per rank at 4096 x 16384).  Returns the result on dst, None elsewhere."""
    if not spectra.is_contiguous():
        raise ValueError("gather_spectra needs contiguous [B, N] spectra")
    return gather_records(spectra, world, rank, dst=dst, group=group, out=out)
