"""StepGraph: one whole training step (zero_grad -> forward -> loss -> backward -> fused AdamW)
captured once as a HIP graph and replayed, instead of ~20 host launches per layer per step.

The reference trains eagerly (`train/train_*.py` train_epoch loops); this is the MI355X
launch path for the launch-bound configurations (w+ latents: 19 tokens, 48 px images:
10 tokens), where host launch cost, not the kernels, sets the step time.

What changes under replay, and how it stays correct:
  * dropout: each captured launch keeps the host seed it was captured with; the library mixes
    a device step counter into every seed (fer_set_step_counter), and the first node of the
    graph advances that counter (fer_step_advance), so every replay draws fresh masks;
  * AdamW: the segment table is uploaded once and the bias-correction step becomes
    host step + *counter (FusedAdamW.freeze_for_graph); hyper-parameters a scheduler changes
    between replays are rewritten into that table before the next replay (sync_graph_hparams);
  * inputs: replays read the tensors captured by the step function -- copy each new batch
    into them (static input buffers), as with any CUDA/HIP graph;
  * memory: activations live in the graph's private pool; the library workspaces are sized by
    the eager warm-up steps, before capture, so no capture-time allocation moves them.
"""
from __future__ import annotations

from typing import Callable, Optional

import torch

from ._lib import check, lib
from . import ops


class StepGraph:
    def __init__(self, step_fn: Callable[[], torch.Tensor], optimizer, warmup: int = 3):
        self.step_fn = step_fn
        self.opt = optimizer
        self.warmup = warmup
        self.graph: Optional[torch.cuda.CUDAGraph] = None
        self.out: Optional[torch.Tensor] = None
        self.counter: Optional[torch.Tensor] = None

    def capture(self) -> "StepGraph":
        dev = torch.device("cuda", torch.cuda.current_device())
        side = torch.cuda.Stream()
        side.wait_stream(torch.cuda.current_stream())
        with torch.cuda.stream(side):  # eager warm-up (sizes every workspace)
            for _ in range(self.warmup):
                self.step_fn()
        torch.cuda.current_stream().wait_stream(side)
        torch.cuda.synchronize()
        # device step counter (uint64 semantics in an int64 tensor)
        self.counter = torch.zeros(1, dtype=torch.int64, device=dev)
        check(lib().fer_set_step_counter(self.counter.data_ptr()), "set_step_counter")
        self.opt.freeze_for_graph(self.counter)
        g = torch.cuda.CUDAGraph()
        # captured on the warm-up stream: the library's per-stream workspaces (ops.WS) sized by
        # the warm-up are the ones the captured launches use (no allocation under capture)
        side.wait_stream(torch.cuda.current_stream())
        # thread_local: a CUDA call from another thread during the capture (RCCL's watchdog querying
        # its events under DDP) must not invalidate it -- with "global" it did, now and then
        # (hipErrorStreamCaptureInvalidated in test_rccl_one_rank_step_graph, profiles/r05u_gpu_tests.txt)
        with torch.cuda.graph(g, stream=side, capture_error_mode="thread_local"):
            check(lib().fer_step_advance(self.counter.data_ptr(), ops.stream()), "step_advance")
            self.out = self.step_fn()
        torch.cuda.current_stream().wait_stream(side)
        self.graph = g
        return self

    def replay(self) -> torch.Tensor:
        """One training step; returns the (device) loss tensor of this replay. A learning-rate
        (or other hyper-parameter) change made since the last replay -- an LR scheduler's
        step -- is written into the captured AdamW segment table first."""
        self.opt.sync_graph_hparams()
        self.graph.replay()
        return self.out

    def release(self) -> None:
        """Back to eager stepping: the optimizer folds the replay count into its host step
        counts (so checkpoints and later eager steps keep the right bias correction)."""
        check(lib().fer_set_step_counter(None), "set_step_counter")
        self.graph = None
        self.opt.unfreeze()
