"""Multi-GPU frame rendering: stratum sharding + one reduce of the accumulator.

The reference is single-GPU (no NCCL/MPI).  Here a frame's strata
(the sqrt(spp) x sqrt(spp) grid of StaticCamera.cpp:74-76, linear index
s_j*sqrt_spp + s_i) are split into contiguous ranges, one per rank; every rank
renders ALL pixels for its range into its own fp64 sum buffer (RT_OUT_SUM), and a
single reduce(sum) to rank 0 combines them — over RCCL/xGMI for GPU ranks, over
gloo for the CPU tests.  The counter-based RNG is keyed by the global stratum
index, so the union of the shards is exactly the one-GPU sample set: the result
equals a single-GPU render up to fp64 summation order.
"""
import torch
import torch.distributed as dist


def strata_shard(n_strata, rank, world):
    """Contiguous stratum range [begin, end) of `rank` (balanced to within one)."""
    if world < 1 or not 0 <= rank < world:
        raise ValueError("bad rank/world")
    return (rank * n_strata // world, (rank + 1) * n_strata // world)


def reduce_frame(acc, dst=0):
    """Sum every rank's accumulator into `dst` (in place on dst)."""
    if dist.is_available() and dist.is_initialized() and dist.get_world_size() > 1:
        dist.reduce(acc, dst=dst, op=dist.ReduceOp.SUM)
    return acc


class ShardedRenderer:
    """Renders one frame per call across the ranks of the default process group.

    render_fn(frame, acc, seed, strata=(begin, count)) must overwrite `acc` with
    the raw per-pixel sums of that stratum range (the Renderer.render_device
    contract with output=RT_OUT_SUM, accumulate=0)."""

    def __init__(self, render_fn, frame, rank=0, world=1):
        self.render_fn = render_fn
        self.frame = frame
        self.rank, self.world = rank, world
        n = frame.sqrt_spp * frame.sqrt_spp
        self.strata = strata_shard(n, rank, world)

    def step(self, acc, seed):
        b, e = self.strata
        self.render_fn(self.frame, acc, seed, (b, e - b))
        return reduce_frame(acc)

    def image(self, acc):
        """Scaled radiance on rank 0 (pixel_samples_scale * sum)."""
        return acc * self.frame.pixel_samples_scale


def max_over_ranks(value, device=None):
    """Max of a float across ranks (the bench's timing rule)."""
    if not (dist.is_available() and dist.is_initialized()) or dist.get_world_size() == 1:
        return float(value)
    t = torch.tensor([float(value)], dtype=torch.float64, device=device)
    dist.all_reduce(t, op=dist.ReduceOp.MAX)
    return float(t.item())
