"""Row-band partitioning of the framebuffer across GPUs and RCCL gather of the shaded bands.

Pixels are independent in the reference's pixel shader (``Default.hlsl:47-161`` reads nothing but its
own fragment and the constants), so a frame splits into horizontal bands with no data exchange while
shading; the one real exchange is assembling the final image on rank 0 (BASELINE config 5:
8192x8192 over 8 GPUs). One process per GPU, ``torch.distributed`` with the ``nccl`` backend
(RCCL over xGMI on MI355X); ``gloo`` runs the same code on CPU tensors for tests.

The G-buffer fill is a function of the global pixel only (``pbr_gbuffer_fill``), so every rank
generates exactly its own rows and the gathered image is bit-identical to a single-GPU frame.
"""
from __future__ import annotations

import datetime
import os
from dataclasses import dataclass
from typing import List, Optional, Tuple

import torch
import torch.distributed as dist


@dataclass(frozen=True)
class Band:
    rank: int
    world: int
    row_begin: int
    row_end: int
    rows_max: int  # rows of the largest band (gather slot height)

    @property
    def rows(self) -> int:
        return self.row_end - self.row_begin


def band_rows(height: int, world: int, rank: int, align: int = 8) -> Band:
    """Rank ``rank``'s rows: equal bands rounded to ``align`` rows (the 8-row shading tile), the
    remainder going to the last ranks so that every band but the tail is tile-aligned."""
    if world < 1 or not 0 <= rank < world or height < 0:
        raise ValueError("bad partition")
    tiles = (height + align - 1) // align
    per, extra = divmod(tiles, world)

    def start(r: int) -> int:
        return min(height, align * (r * per + max(0, r - (world - extra))))

    r0, r1 = start(rank), start(rank + 1)
    rows_max = min(height, align * (per + (1 if extra else 0)))
    return Band(rank, world, r0, r1, rows_max)


def all_bands(height: int, world: int, align: int = 8) -> List[Band]:
    return [band_rows(height, world, r, align) for r in range(world)]


# Failure detection (the reference polls GetDeviceRemovedReason around every Draw step,
# PBRApp.cpp:247): the band gather gives up after PBR_DIST_TIMEOUT_S seconds instead of blocking on a dead peer until
# the backend's default (30 min). It runs on its own process group (gather_group) created with that timeout; RCCL's
# watchdog then aborts the communicator and the process exits non-zero, gloo raises, and BandGather.wait turns that
# into GatherError. The default group -- the rendezvous, barriers, the bench's max-over-ranks all-reduce -- waits at
# least RENDEZVOUS_TIMEOUT_S, so that ranks whose interpreters start seconds apart (each imports torch first) still
# meet even when the gather timeout is short.
DEFAULT_TIMEOUT_S = 300.0
RENDEZVOUS_TIMEOUT_S = 120.0


class GatherError(RuntimeError):
    """A band gather (or another collective) failed: a peer died, or it did not answer within the timeout."""


def collective_timeout() -> datetime.timedelta:
    """The band gather's timeout: PBR_DIST_TIMEOUT_S seconds (default DEFAULT_TIMEOUT_S)."""
    return datetime.timedelta(seconds=float(os.environ.get("PBR_DIST_TIMEOUT_S", DEFAULT_TIMEOUT_S)))


def init_from_env(backend: str, always: bool = False, timeout: Optional[datetime.timedelta] = None
                  ) -> Tuple[int, int, int]:
    """(rank, world, local_rank) from torchrun's environment; initialises the default group once: at
    world > 1, and at world 1 too when ``always`` (so a single-rank run exercises the same RCCL
    communicator init / teardown and collectives as the multi-GPU one). ``timeout`` (default: the larger of
    collective_timeout() and RENDEZVOUS_TIMEOUT_S) bounds the rendezvous and the default group's collectives.
    Rendezvous: PBR_DIST_INIT_METHOD when set (e.g. ``file:///tmp/run/rdzv``, a file store that needs no free TCP
    port), else MASTER_ADDR / MASTER_PORT (env://)."""
    rank = int(os.environ.get("RANK", "0"))
    world = int(os.environ.get("WORLD_SIZE", "1"))
    local = int(os.environ.get("LOCAL_RANK", "0"))
    if (world > 1 or always) and not dist.is_initialized():
        if timeout is None:
            timeout = max(collective_timeout(), datetime.timedelta(seconds=RENDEZVOUS_TIMEOUT_S))
        kwargs = {"timeout": timeout}
        method = os.environ.get("PBR_DIST_INIT_METHOD")
        if method:
            kwargs["init_method"] = method
        else:
            os.environ.setdefault("MASTER_ADDR", "127.0.0.1")
            os.environ.setdefault("MASTER_PORT", "29517")
        if backend == "nccl":
            kwargs["device_id"] = torch.device("cuda", local)  # one GPU per rank (RCCL)
        dist.init_process_group(backend=backend, rank=rank, world_size=world, **kwargs)
    return rank, world, local


_gather_group = None  # (the default group it was created under, the gather group)


def gather_group():
    """The process group the band gather runs on: every rank, with collective_timeout() (created once per default
    process group, collectively: every rank calls it the first time it builds a BandGather). None at world 1. The
    cache is keyed on the default group object, so after destroy_process_group() and a new init_process_group() the
    next BandGather builds a group of the new world instead of reusing one of the destroyed world."""
    global _gather_group
    if not dist.is_initialized() or dist.get_world_size() <= 1:
        return None
    world = dist.group.WORLD
    if _gather_group is None or _gather_group[0] is not world:
        _gather_group = (world, dist.new_group(timeout=collective_timeout()))
    return _gather_group[1]


class BandGather:
    """Gathers every rank's (rows_max, W, 4) band into rank 0's (world, rows_max, W, 4) buffer.

    Implemented as one grouped point-to-point round (each peer sends its band straight to rank 0
    over its own xGMI link; rank 0 posts one receive per peer) rather than a ring all-gather: only
    rank 0 needs the image, and a star puts all 7 links into rank 0 to work at once.
    """

    def __init__(self, band: Band, width: int, device, group=None, dtype=torch.float32):
        self.band = band
        self.group = group if group is not None else gather_group()
        self.width = width
        self.frame: Optional[torch.Tensor] = None
        if band.rank == 0:
            self.frame = torch.empty((band.world, band.rows_max, width, 4), dtype=dtype, device=device)
        # gloo cannot move device tensors point to point: stage through host memory (tests only;
        # the benchmark's multi-GPU path is RCCL).
        self.host_staged = (band.world > 1 and torch.device(device).type == "cuda"
                            and dist.get_backend(self.group) == "gloo")

    def start(self, band_out: torch.Tensor):
        """Post the gather of ``band_out`` ((rows_max, W, 4)); returns the list of work handles."""
        b = self.band
        if b.world == 1:
            self.frame[0].copy_(band_out, non_blocking=True)
            return []
        if self.host_staged:
            self._gather_host_staged(band_out)
            return []
        if b.rank == 0:
            self.frame[0].copy_(band_out)
            ops = [dist.P2POp(dist.irecv, self.frame[r], r, self.group) for r in range(1, b.world)]
        else:
            ops = [dist.P2POp(dist.isend, band_out, 0, self.group)]
        return dist.batch_isend_irecv(ops)

    def _gather_host_staged(self, band_out: torch.Tensor) -> None:
        b = self.band
        if b.rank == 0:
            self.frame[0].copy_(band_out)
            bufs = [torch.empty(tuple(band_out.shape), dtype=band_out.dtype) for _ in range(1, b.world)]
            works = [dist.irecv(buf, r, self.group) for r, buf in zip(range(1, b.world), bufs)]
            BandGather.wait(works)
            for r, buf in zip(range(1, b.world), bufs):
                self.frame[r].copy_(buf)
        else:
            try:
                dist.send(band_out.cpu(), 0, self.group)
            except RuntimeError as e:
                raise GatherError(f"rank {b.rank}: sending its band to rank 0 failed: {e}") from e

    @staticmethod
    def wait(handles) -> None:
        """Wait for posted gather work; a failure (a dead peer, or no answer within the process group's
        timeout) raises GatherError naming it."""
        for h in handles:
            try:
                h.wait()
            except RuntimeError as e:
                raise GatherError(f"band gather failed (peer lost or timed out; PBR_DIST_TIMEOUT_S="
                                  f"{collective_timeout().total_seconds():g}): {e}") from e

    def assembled(self, height: int) -> Optional[torch.Tensor]:
        """Rank 0: the (height, W, 4) image stitched from the gathered slots (a copy when bands are
        uneven, else a view)."""
        if self.frame is None:
            return None
        bands = all_bands(height, self.band.world)
        if all(b.rows == self.band.rows_max for b in bands):
            return self.frame.reshape(-1, self.width, 4)[:height]
        return torch.cat([self.frame[b.rank, : b.rows] for b in bands], dim=0)
