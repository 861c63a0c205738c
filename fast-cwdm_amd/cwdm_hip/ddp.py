"""Data-parallel gradient averaging overlapped with the native backward.

The native U-Net backward runs in segments (output head, each ResBlock in
reverse, then conv_in + time_embed; cwdm_unet_segment_range).  Each finished
segment's gradient range is adjacent to (and below) the previous one in the
flat buffer, so the reducer grows one contiguous pending range and launches an
async all-reduce (RCCL over xGMI with the "nccl" backend, gloo on CPU) as soon
as it reaches ``bucket_bytes``; later segments keep computing on the compute
stream while the collective runs beside them (issued from the reducer's own
stream).  At the end every launched collective is waited on (stream-ordered,
no host sync) and the buffer is divided by the world size.  Buckets default to
64 MB: big enough that a ring all-reduce over point-to-point xGMI links is bandwidth- not
latency-bound, small enough that ~5 buckets overlap the 81.5 M-parameter
backward.
"""
import torch
import torch.distributed as dist


class GradBucketReducer:
    """``force``: run the collectives even at world size 1 (tests exercise the
    RCCL path on a one-GPU box that way).  ``timing``: record HIP events per
    bucket (launch on the compute stream, start / end on the communicator
    stream) and at the end of the backward, read back by ``timeline()``.

    GPU buffers: each bucket's all-reduce is issued from the reducer's own
    stream, which first waits for the bucket's gradients on the compute stream
    (an event); RCCL's internal stream then waits on that stream, and
    ``work.wait()`` makes the reducer stream wait for the collective, so the
    end event marks its completion.  At the end the compute stream waits for
    the reducer stream (no host sync)."""

    def __init__(self, group=None, bucket_bytes=64 << 20, force=False, timing=False):
        self.group = group
        self.bucket = max(int(bucket_bytes) // 4, 1)
        self.force = force
        self.timing = timing
        self.launched = 0
        self._works = []
        self._lo = self._hi = None
        self._stream = None
        self._events = []       # per bucket: (ready on compute, start on comm, end on comm)
        self._t0 = self._bwd_end = None
        self._active = False    # inside a backward (between its first segment and the end call)

    @property
    def world(self):
        return dist.get_world_size(self.group) if dist.is_initialized() else 1

    def _event(self):
        return torch.cuda.Event(enable_timing=self.timing)

    def _flush(self, flat):
        if self._lo is not None and self._hi > self._lo:
            buf = flat[self._lo:self._hi]
            if buf.is_cuda:
                if self._stream is None:
                    self._stream = torch.cuda.Stream(device=buf.device)
                ready = self._event()
                ready.record()                       # the bucket's gradients are done on the compute stream
                with torch.cuda.stream(self._stream):
                    self._stream.wait_event(ready)
                    start = self._event()
                    start.record()
                    work = dist.all_reduce(buf, group=self.group, async_op=True)
                    work.wait()                      # the reducer stream waits for RCCL's stream
                    end = self._event()
                    end.record()
                self._events.append((ready, start, end))
            else:
                self._works.append(dist.all_reduce(buf, group=self.group, async_op=True))
            self.launched += 1
        self._lo = self._hi = None

    def __call__(self, seg, flat, off, n):
        """UNetModel._grad_hook: (seg, flat grad buffer, offset, count); seg None = end."""
        if self.world == 1 and not (self.force and dist.is_initialized()):
            return
        if not self._active:
            self._active = True
            self._events = []   # this backward's buckets only (the reducer lives across steps)
            self._t0 = self._bwd_end = None
        if seg is None:
            self._active = False
            self._flush(flat)
            if flat.is_cuda:
                if self.timing:
                    self._bwd_end = self._event()
                    self._bwd_end.record()
                if self._stream is not None:
                    torch.cuda.current_stream().wait_stream(self._stream)
            for w in self._works:
                w.wait()
            self._works = []
            flat.div_(self.world)
            return
        if self.timing and self._t0 is None and flat.is_cuda:
            self._t0 = self._event()
            self._t0.record()                        # after the first segment
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

    def timeline(self):
        """(backward_end_ms, [(ready_ms, start_ms, end_ms) per bucket]) relative
        to the end of the first backward segment; synchronises.  A bucket whose
        start precedes backward_end ran beside the backward.  None when no
        backward was timed (timing off, or world size 1 without force)."""
        if getattr(self, "_t0", None) is None or getattr(self, "_bwd_end", None) is None:
            return None
        torch.cuda.synchronize()
        ms = lambda e: self._t0.elapsed_time(e)  # noqa: E731
        return ms(self._bwd_end), [(ms(r), ms(s), ms(e)) for r, s, e in self._events]


def broadcast_params(params, src=0, group=None):
    """Start every rank from rank ``src``'s weights."""
    if not dist.is_initialized() or dist.get_world_size(group) == 1:
        return
    with torch.no_grad():
        for p in params:
            dist.broadcast(p.data, src, group=group)
            torch.autograd.graph.increment_version(p)
