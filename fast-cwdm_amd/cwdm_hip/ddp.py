"""Data-parallel gradient averaging overlapped with the native backward.

The native U-Net backward runs in segments (output head, each ResBlock in
reverse, then conv_in + time_embed; cwdm_unet_segment_range).  Each finished
segment's gradient range is adjacent to (and below) the previous one in the
flat buffer, so the reducer grows one contiguous pending range and launches an
async all-reduce (RCCL over xGMI with the "nccl" backend, gloo on CPU) as soon
as it reaches ``bucket_bytes``; later segments keep computing on the compute
stream while the collective runs on the communicator's stream.  At the end
every launched collective is waited on (stream-ordered, no host sync) and the
buffer is divided by the world size.  Buckets default to 64 MB: big enough
that a ring all-reduce over point-to-point xGMI links is bandwidth- not
latency-bound, small enough that ~5 buckets overlap the 81.5 M-parameter
backward.
"""
import torch
import torch.distributed as dist


class GradBucketReducer:
    """``force``: run the collectives even at world size 1 (tests exercise the
    RCCL path on a one-GPU box that way)."""

    def __init__(self, group=None, bucket_bytes=64 << 20, force=False):
        self.group = group
        self.bucket = max(int(bucket_bytes) // 4, 1)
        self.force = force
        self.launched = 0
        self._works = []
        self._lo = self._hi = None

    @property
    def world(self):
        return dist.get_world_size(self.group) if dist.is_initialized() else 1

    def _flush(self, flat):
        if self._lo is not None and self._hi > self._lo:
            self._works.append(dist.all_reduce(flat[self._lo:self._hi], group=self.group, async_op=True))
            self.launched += 1
        self._lo = self._hi = None

    def __call__(self, seg, flat, off, n):
        """UNetModel._grad_hook: (seg, flat grad buffer, offset, count); seg None = end."""
        if self.world == 1 and not (self.force and dist.is_initialized()):
            return
        if seg is None:
            self._flush(flat)
            for w in self._works:
                w.wait()
            self._works = []
            flat.div_(self.world)
            return
        if self._lo is None:
            self._lo, self._hi = off, off + n
        elif off + n == self._lo:
            self._lo = off
        elif off == self._hi:
            self._hi = off + n
        else:
            self._flush(flat)
            self._lo, self._hi = off, off + n
        if self._hi - self._lo >= self.bucket:
            self._flush(flat)


def broadcast_params(params, src=0, group=None):
    """Start every rank from rank ``src``'s weights."""
    if not dist.is_initialized() or dist.get_world_size(group) == 1:
        return
    with torch.no_grad():
        for p in params:
            dist.broadcast(p.data, src, group=group)
            torch.autograd.graph.increment_version(p)
