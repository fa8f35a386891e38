"""Long-term feature bank (LFB) extraction — the loop of generate_evp_LFB.py:439-520, MI355X build.

The reference: DataLoader(batch 200, 8 workers, PIL decode + Resize/CenterCrop/ToTensor/Normalize on
the host, generate_evp_LFB.py:389-410) -> ``.to(device)`` -> ``model.forward(..., return_features=True)``
-> ``.data.cpu().numpy()`` -> ``np.concatenate`` onto a float64 array after every batch (quadratic host
copying, :457/477/497) -> pickle (:513-520), which ``tecno.py`` / ``trans_SV_output.py`` load back
(tecno.py:80-85).

Here (``extract_lfb``):

* the host only decodes: dataset items are the DECODED uint8 frame / segmap [H, W, 3] and the raw RAFT
  flow [h, w, 2] f32 (``CholecFlowDataset(..., decoded=True)``), batched by DataLoader workers into
  pinned memory — 4x fewer bytes over PCIe than the reference's normalised f32 tensors;
* a copy stream moves batch k+1 host -> HBM while batch k computes (two device slots, events);
* on the compute stream the GPU transforms (svk.preproc.frame_transform / flow_transform: Pillow-exact
  Resize(250) + CenterCrop(224) + Normalize, cv2-exact flow resize + rescale + crop) write straight into
  the static input buffers of the extraction forward, which replays as ONE HIP graph per batch
  (svk.graphs.GraphedForward);
* each batch's [B, 2048] features go to a preallocated device bank, and from there asynchronously
  (a third stream) into a preallocated pinned host bank — no growing arrays;
* frames are sharded across ranks (one process per GPU, contiguous index shards, svk.shard) and
  gathered at the end.

Datasets whose items are already-transformed tensors (the reference's own transform pipeline) run the
same loop without the GPU transform step (their f32 tensors are copied in as they are).
``save_lfb`` writes the reference's pickle format (float64 ndarray) plus an fp32 ``.npy`` sidecar.
"""
import pickle

import numpy as np
import torch

from ._lib import SvkError
from .shard import shard_range, gather_rows

FEAT = 2048


def _is_decoded(item):
    img = item[0]
    return (isinstance(img, np.ndarray) and img.dtype == np.uint8) or \
        (isinstance(img, torch.Tensor) and img.dtype == torch.uint8)


class _Slot:
    """One device-side input slot of the double-buffered pipeline."""

    def __init__(self):
        self.bufs = None
        self.ready = torch.cuda.Event()
        self.free = torch.cuda.Event()
        self.host = None           # the host batch whose copy into this slot may still be in flight


def _loader(dataset, a, b, batch_size, num_workers):
    from torch.utils.data import DataLoader, Subset
    sub = Subset(dataset, range(a, b))
    return DataLoader(sub, batch_size=batch_size, shuffle=False, num_workers=num_workers,
                      pin_memory=True, drop_last=False, persistent_workers=False)


class LFBExtractor:
    """The pipelined extraction loop over one model (state kept across calls: device slots, the static
    graph inputs, the captured graph, the streams)."""

    def __init__(self, model, batch_size=256, device=None, graph=True):
        if model.training:
            raise SvkError("extract_lfb: eval-mode model expected (generate_evp_LFB.py:437 calls model.eval())")
        self.model, self.B, self.graph = model, int(batch_size), graph
        self.device = device or torch.device("cuda", torch.cuda.current_device())
        d = self.device
        self.static = (torch.empty(self.B, 1, 3, 224, 224, device=d), torch.empty(self.B, 1, 3, 224, 224, device=d),
                       torch.empty(self.B, 1, 2, 224, 224, device=d))
        self.h2d, self.d2h = torch.cuda.Stream(device=d), torch.cuda.Stream(device=d)
        self.slots = [_Slot(), _Slot()]
        self.gf = None
        self.k = 0

    def _stage(self, batch, decoded):
        """Batch k: host -> HBM on the copy stream (slot k % 2), then the GPU transforms into the static
        graph inputs on the compute stream.  Returns the number of frames."""
        img, seg, flow = batch[0], batch[1], batch[2]
        bsz, B, comp = img.shape[0], self.B, torch.cuda.current_stream(self.device)
        if bsz > B:
            raise SvkError(f"extract_lfb: batch of {bsz} frames larger than batch_size {B}")
        sl = self.slots[self.k % 2]
        self.k += 1
        if sl.host is not None:
            sl.ready.synchronize()                    # the previous copy out of the old host batch has run
        self.h2d.wait_event(sl.free)                  # the compute stream no longer reads this slot
        with torch.cuda.stream(self.h2d):
            srcs = (img, seg, flow)
            if sl.bufs is None or any(t.shape[1:] != s.shape[1:] or t.dtype != s.dtype for t, s in zip(srcs, sl.bufs)):
                sl.bufs = tuple(torch.empty((B,) + tuple(t.shape[1:]), dtype=t.dtype, device=self.device) for t in srcs)
            for dst, src in zip(sl.bufs, srcs):
                dst[:bsz].copy_(src, non_blocking=True)
            sl.ready.record(self.h2d)
        sl.host = batch
        comp.wait_event(sl.ready)
        x, y, fl = self.static
        if decoded:
            from .preproc import frame_transform, flow_transform
            frame_transform(sl.bufs[0][:bsz], out=x.view(B, 3, 224, 224)[:bsz])
            frame_transform(sl.bufs[1][:bsz], out=y.view(B, 3, 224, 224)[:bsz])
            flow_transform(sl.bufs[2][:bsz], out=fl.view(B, 2, 224, 224)[:bsz])
        else:
            x.view(B, 3, 224, 224)[:bsz].copy_(sl.bufs[0][:bsz].view(bsz, 3, 224, 224))
            y.view(B, 3, 224, 224)[:bsz].copy_(sl.bufs[1][:bsz].view(bsz, 3, 224, 224))
            fl.view(B, 2, 224, 224)[:bsz].copy_(sl.bufs[2][:bsz].view(bsz, 2, 224, 224))
        sl.free.record(comp)
        return bsz

    def _forward(self):
        x, y, fl = self.static
        if not self.graph:
            return self.model(x, y, fl, return_features=True)
        if self.gf is None:
            from .graphs import GraphedForward
            self.gf = GraphedForward(self.model, x, y, fl, return_features=True)
        return self.gf()

    def run(self, batches, n, to_host=True, decoded=None):
        """Features of the ``n`` frames in ``batches`` (collated (frame, segmap, flow, ...) tensors) ->
        (n, 2048) f32: pinned host memory if ``to_host`` (async per-batch D2H), else on the device."""
        dev_bank = torch.empty(n, FEAT, dtype=torch.float32, device=self.device)
        host_bank = torch.empty(n, FEAT, dtype=torch.float32, pin_memory=True) if to_host else None
        comp = torch.cuda.current_stream(self.device)
        row = 0
        with torch.no_grad():
            for batch in batches:
                if decoded is None:
                    decoded = batch[0].dtype == torch.uint8
                bsz = self._stage(batch, decoded)
                if row + bsz > n:
                    raise SvkError(f"extract_lfb: more than the {n} frames announced")
                out = self._forward()
                dev_bank[row:row + bsz].copy_(out[:bsz])
                if to_host:
                    self.d2h.wait_stream(comp)
                    with torch.cuda.stream(self.d2h):
                        host_bank[row:row + bsz].copy_(dev_bank[row:row + bsz], non_blocking=True)
                row += bsz
            if row != n:
                raise SvkError(f"extract_lfb: got {row} frames, expected {n}")
            self.d2h.synchronize()
            comp.synchronize()
        return host_bank if to_host else dev_bank


def extract_lfb(model, dataset=None, batch_size=256, device=None, rank=0, world=1, group=None, num_workers=8,
                batches=None, n=None, graph=True, to_host=True):
    """Run ``model(x, y, flow, return_features=True)`` over the frames in index order and return the
    (N, 2048) float32 bank (pinned host memory if ``to_host``, else on the device; the full bank on every
    rank when world > 1).

    ``dataset``: items (frame, segmap, flow, ...) — decoded uint8 [H, W, 3] / [H, W, 3] / raw f32 [h, w, 2]
    (the fast path: ``CholecFlowDataset(..., decoded=True)``) or the reference's transformed f32
    [3, 224, 224] / [3, 224, 224] / [2, 224, 224]; read through a DataLoader (``num_workers`` decode
    processes, pinned batches) over this rank's contiguous shard.  ``batches`` instead: an iterable of
    already-collated batches covering ``n`` frames of this rank's shard."""
    ex = LFBExtractor(model, batch_size, device, graph)
    total = None
    if batches is None:
        if dataset is None:
            raise SvkError("extract_lfb: give a dataset or an iterable of batches")
        total = len(dataset)
        a, b = shard_range(total, rank, world)
        batches = _loader(dataset, a, b, batch_size, num_workers) if b > a else []
        n = b - a
    elif n is None:
        raise SvkError("extract_lfb: n (frames in the given batches) is required with batches=")
    bank = ex.run(batches, int(n), to_host=to_host and world == 1)
    if world > 1:
        full = gather_rows(bank, total if total is not None else int(n) * world, group)
        return full.cpu().pin_memory() if to_host else full
    return bank


def save_lfb(bank, pkl_path, npy_path=None):
    """Reference format: pickle of a float64 (N, 2048) ndarray (generate_evp_LFB.py:513-520)."""
    arr = bank.detach().cpu().numpy()
    with open(pkl_path, "wb") as f:
        pickle.dump(arr.astype(np.float64), f)
    if npy_path:
        np.save(npy_path, arr.astype(np.float32))
