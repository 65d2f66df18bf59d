"""Batched flow inference: the evaluate / demo path at large batch, optionally as one hipGraph.

Reference: `evaluate.py:95-127` (``validate_sintel``: InputPadder('sintel') -> ``model(image1,
image2, iters=32, test_mode=True)`` -> unpad) and `core/raft.py:141-142` (test-mode outputs).  The
reference runs one pair at a time and re-issues every kernel of the 32-iteration GRU loop from
Python.  On MI355X:

* pairs are batched (288 GB HBM holds hundreds of Sintel-size pairs with the on-the-fly
  correlation, tens with the all-pairs pyramid);
* test mode skips the convex upsample AND the mask head of every iteration but the last (the
  reference computes and discards both, `core/raft.py:133-142`; outputs are identical);
* ``graph=True`` captures the whole padded forward (encoders, correlation, the GRU loop, the final
  upsample) into a single hipGraph on static input buffers: one ``hipGraphLaunch`` replaces
  ~30 launches per iteration x 32 iterations of host issue.  Replays are bitwise identical to
  the eager run (same kernels, same buffers).
"""
import torch

from ..utils.utils import InputPadder


class FlowInference:
    """``FlowInference(model, iters=32)(image1, image2) -> (flow_low, flow_up)`` in test mode.

    Images are float 0..255 (B, 3, H, W) on the model's device, any H, W (padded to a multiple of
    8 with ``pad_mode`` as `core/utils/utils.py:7-24`; outputs are un-padded).  With ``graph=True``
    the first call for a given input shape captures a hipGraph; later calls with the same shape
    copy into the static inputs and replay it.
    """

    def __init__(self, model, iters=32, pad_mode='sintel', graph=False, warmup=1):
        self.model = model
        self.iters = int(iters)
        self.pad_mode = pad_mode
        self.graph = bool(graph)
        self.warmup = int(warmup)
        self._g = None
        self._key = None

    def _device(self):
        return next(self.model.parameters()).device

    def _forward(self, i1, i2, flow_init=None):
        return self.model(i1, i2, iters=self.iters, flow_init=flow_init, test_mode=True)

    def _capture(self, i1, i2, flow_init):
        self._s1 = i1.clone()
        self._s2 = i2.clone()
        self._sf = None if flow_init is None else flow_init.clone()
        side = torch.cuda.Stream(device=i1.device)
        side.wait_stream(torch.cuda.current_stream(i1.device))
        with torch.cuda.stream(side):
            for _ in range(max(1, self.warmup)):  # allocator warm-up / autotune outside capture
                self._forward(self._s1, self._s2, self._sf)
        torch.cuda.current_stream(i1.device).wait_stream(side)
        torch.cuda.synchronize(i1.device)
        self._g = torch.cuda.CUDAGraph()
        with torch.cuda.graph(self._g):
            self._out = self._forward(self._s1, self._s2, self._sf)
        self._key = self._shape_key(i1, flow_init)

    @staticmethod
    def _shape_key(i1, flow_init):
        return (tuple(i1.shape), i1.dtype, i1.device,
                None if flow_init is None else tuple(flow_init.shape))

    @torch.no_grad()
    def __call__(self, image1, image2, flow_init=None):
        """``flow_init``: optional (B, 2, H/8, W/8) warm start at 1/8 of the PADDED size
        (`core/raft.py:119-120`; the reference's warm-start evaluation, `evaluate.py:31-41`)."""
        padder = InputPadder(image1.shape, mode=self.pad_mode)
        i1, i2 = padder.pad(image1, image2)
        if self.graph and i1.is_cuda:
            if self._key != self._shape_key(i1, flow_init):
                self._capture(i1.contiguous(), i2.contiguous(), flow_init)
            self._s1.copy_(i1)
            self._s2.copy_(i2)
            if flow_init is not None:
                self._sf.copy_(flow_init)
            self._g.replay()
            flow_low, flow_up = self._out
            flow_low, flow_up = flow_low.clone(), flow_up.clone()
        else:
            flow_low, flow_up = self._forward(i1, i2, flow_init)
        return flow_low, padder.unpad(flow_up)
