"""Host-batch staging for the unchanged `main.py` loop (TRANSFORMER.train_step with CPU tensors).

The reference moves each DataLoader batch with a synchronous pageable `.to(DEVICE)` on the compute
stream before the step (core/models.py:120-122; batches from core/dataset.py:8-29).  Here a batch
goes host -> pinned slot (CPU copy) -> device ring slot on a side copy stream, overlapped with the
previous step's kernels, and the step reads it through the engine's indexed entry point
(capgen_train_step_indexed) so every pointer the captured step graph holds stays fixed:

  * two pinned slots and a device ring of 2 B images (features f32, positions f32, captions);
  * slot s is rewritten (host) only after its previous H2D finished, and its device copy is
    overwritten (copy stream) only after the step that read it finished (`consumed[s]`);
  * the compute stream waits for slot s's H2D, copies the slot's image indices and captions
    into the two fixed device buffers the graph reads (two small D2D copies), runs the step.

Features stay f32 on the device (the engine's pack kernel converts while gathering), so the host
does no dtype conversion.
"""
from __future__ import annotations

import torch


class HostBatchStager:
    SLOTS = 2

    def __init__(self, device, B: int, N: int, F: int, P: int, T: int):
        self.device = torch.device(device)
        self.shape = (B, N, F, P, T)
        S = self.SLOTS
        self.pin_f = [torch.empty((B, N, F), dtype=torch.float32, pin_memory=True) for _ in range(S)]
        self.pin_p = [torch.empty((B, N, P), dtype=torch.float32, pin_memory=True) for _ in range(S)]
        self.pin_c = [torch.empty((B, T), dtype=torch.int32, pin_memory=True) for _ in range(S)]
        dev = self.device
        self.store_f = torch.empty((S * B, N, F), dtype=torch.float32, device=dev)
        self.store_p = torch.empty((S * B, N, P), dtype=torch.float32, device=dev)
        self.caps_ring = torch.empty((S, B, T), dtype=torch.int32, device=dev)
        self.idx_slot = [torch.arange(s * B, (s + 1) * B, dtype=torch.int32, device=dev) for s in range(S)]
        self.caps = torch.empty((B, T), dtype=torch.int32, device=dev)  # fixed pointers for the graph
        self.idx = torch.empty((B,), dtype=torch.int32, device=dev)
        self.copy_stream = torch.cuda.Stream(dev)
        # A stager replaces another when the batch shape changes (main.py's last, smaller batch of an
        # epoch): the buffers above may reuse memory the caching allocator got back from the old
        # stager while a step issued on the current stream may still read it.  Every H2D of this
        # stager runs on copy_stream, so make it wait for everything issued so far on that stream.
        self.copy_stream.wait_stream(torch.cuda.current_stream(dev))
        self.h2d_done = [torch.cuda.Event() for _ in range(S)]
        self.consumed = [torch.cuda.Event() for _ in range(S)]
        self.i = 0

    def fits(self, feats, pos, caps) -> bool:
        B, N, F, P, T = self.shape
        return (tuple(feats.shape) == (B, N, F) and tuple(pos.shape) == (B, N, P)
                and tuple(caps.shape) == (B, T))

    def stage(self):
        """Slot index for the next batch; waits (host) until its pinned buffers are free."""
        s = self.i % self.SLOTS
        self.h2d_done[s].synchronize()  # a never-recorded event returns at once
        return s

    def run(self, engine, feats, pos, caps):
        """Stage one host batch and run engine.train_step_indexed on it (current stream)."""
        s = self.stage()
        B = self.shape[0]
        self.pin_f[s].copy_(torch.as_tensor(feats))
        self.pin_p[s].copy_(torch.as_tensor(pos))
        self.pin_c[s].copy_(torch.as_tensor(caps))
        cur = torch.cuda.current_stream(self.device)
        with torch.cuda.stream(self.copy_stream):
            self.copy_stream.wait_event(self.consumed[s])  # the step that read ring slot s is done
            self.store_f[s * B:(s + 1) * B].copy_(self.pin_f[s], non_blocking=True)
            self.store_p[s * B:(s + 1) * B].copy_(self.pin_p[s], non_blocking=True)
            self.caps_ring[s].copy_(self.pin_c[s], non_blocking=True)
            self.h2d_done[s].record(self.copy_stream)
        cur.wait_event(self.h2d_done[s])
        self.idx.copy_(self.idx_slot[s], non_blocking=True)
        self.caps.copy_(self.caps_ring[s], non_blocking=True)
        out = engine.train_step_indexed(self.store_f, self.store_p, self.idx, self.caps)
        self.consumed[s].record(cur)
        self.i += 1
        return out
