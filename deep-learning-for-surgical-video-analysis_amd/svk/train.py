"""Native frozen-backbone training step of MixVisionTransformerEVP — MI355X build.

Replaces the inner loop of ``train_model`` (train_evp.py:473-515): autocast forward, CE(sum) +
SmoothL1(sum) loss, backward, SGD step.  Every op is an svk kernel with an explicit backward:

* what trains (train_evp.py:379-382): parameters whose names contain ``head``, ``prompt``,
  ``flow_encoder``, ``cross_attn_s3`` or ``cross_attn_s4`` (24.79 M for mit_b2_evp).  The
  backbone is frozen but the prompts are injected before every block, so the backward runs the
  *data* gradient through every backbone block (no weight gradients there);
* train-mode semantics: timm DropPath per block branch (drop_path_rate 0.1, linear rule,
  mix_transformer_evp.py:238) fused as a per-frame row scale into the branch GEMM epilogue and its
  adjoint; Dropout2d(0.1) on the fused head map applied after the (linear) average pool;
  BatchNorm with batch statistics (head linear_fuse.bn, flow encoder bn1..4) and the running-stat
  momentum update;
* the head is NOT folded in training (its BN uses batch statistics): linear_c* run on the 7x7
  resized maps (exact: resize and the per-token Linear commute) into one [B*49, 8192] buffer,
  then the 1x1 fuse GEMM, BN, ReLU, pool;
* parameters live in one flat f32 buffer (the nn.Parameters are views into it, their ``.grad``
  views into a flat gradient buffer), so SGD is one kernel, the DDP gradient all-reduce is one
  RCCL call on one buffer, and a single batched gather re-packs every compute-dtype weight
  view (forward and transposed layouts) after the step;
* GradScaler (train_evp.py:443, 512-515) is not needed: bf16 has fp32's exponent range.

Frames per step B = 88 at the reference setting (train_evp.py:28).
"""
import os

import numpy as np
import torch
from torch.autograd.graph import increment_version

from . import ops
from ._lib import SvkError
from .pack import pad_channels, conv_w, conv_w_s2d

# MixFFN front half of the training forward through svk_mixffn_fc1_dwconv_ex (A/B switch; channel widths it
# is used for: stages 1-2 by default, "64,128,320,512" adds stages 3-4)
TRAIN_FC1_DWCONV = os.environ.get("SVK_TRAIN_FC1_DWCONV", "1") == "1"
# sequence-reduction conv data gradient as GEMM + vectorised scatter-add (A/B switch; 0 = fused scatter epilogue)
TRAIN_UNPATCHIFY_SPLIT = os.environ.get("SVK_TRAIN_UNPATCHIFY_SPLIT", "1") == "1"
# conv data gradients (frozen patch embeds, handcrafted-prompt convs) as per-tap GEMM + col2im gather (A/B
# switch; 0 = the transposed-conv gather GEMM over input pixels)
TRAIN_COL2IM = os.environ.get("SVK_TRAIN_COL2IM", "1") == "1"
# stages 3-4 (14 x 14 / C = 320, 7 x 7 / C = 512): the frozen DWConv + fc1 data gradient as ONE kernel — the
# matrix-core dw_fc2 with flipped taps, no activation and W1ᵀ in place of W2 — instead of dwconv3x3 + GEMM
TRAIN_DWFC_BWD = os.environ.get("SVK_TRAIN_DWFC_BWD", "1") == "1"
# the step's DropPath masks in one launch (svk_keep_mask_multi) instead of one keep_mask launch per mask
TRAIN_MASK_MULTI = os.environ.get("SVK_TRAIN_MASK_MULTI", "1") == "1"
# stages 3-4 training forward: DWConv + GELU + fc2 (+ DropPath scale + residual) as one matrix-core dw_fc2 launch
# that also stores the GELU pre-activation (round 6), instead of dwconv3x3(pre_out) + GEMM.  Parity-tested but OFF:
# at B = 88 its one-tile-per-workgroup grid (352 workgroups for 512 slots) ran the step 0.3 % slower
# (profiles/r06/train_dwfc_fwd_ab.txt: 6 157 / 6 166 vs 6 181 / 6 178 frames/s, interleaved, same box)
TRAIN_DWFC_FWD = os.environ.get("SVK_TRAIN_DWFC_FWD", "0") == "1"
TRAIN_FC1_DWCONV_C = tuple(int(c) for c in os.environ.get("SVK_TRAIN_FC1_DWCONV_C", "32,64,128").split(","))

TRAINABLE = ("head", "prompt", "flow_encoder", "cross_attn_s3", "cross_attn_s4")
_BN_BUFFERS = ("running_mean", "running_var", "num_batches_tracked")
DROP_PATH_RATE = 0.1
HEAD_DROPOUT = 0.1
BLOCK_EPS, LN_EPS, BN_EPS, BN_MOMENTUM = 1e-6, 1e-5, 1e-5, 0.1

_DESC = np.dtype([("src", "<i8"), ("dst", "<i8"), ("n", "<i4", 4), ("s", "<i8", 4), ("lim", "<i4", 4),
                  ("start", "<i8")])      # csrc/train.hip PackDesc
_TILE = np.dtype([("src", "<i8"), ("dst", "<i8"), ("K", "<i4"), ("N", "<i4"), ("n0", "<i4"),
                  ("k0", "<i4")])         # csrc/train.hip PackTile
# transposed weight packs through the tiled transpose kernel (A/B switch; 0 = the generic strided gather)
PACK_TRANSPOSE = os.environ.get("SVK_PACK_TRANSPOSE", "1") == "1"
# the generic gather 8 elements per thread (svk_pack_params8; 0 = one element per thread)
PACK_PARAMS8 = os.environ.get("SVK_PACK_PARAMS8", "1") == "1"
# conv data-gradient packs (.D) through the tiled transpose (A/B switch; 0 = the strided gather)
PACK_D_TRANSPOSE = os.environ.get("SVK_PACK_D_T", "1") == "1"


def is_trainable(name):
    return any(k in name for k in TRAINABLE) and not name.endswith(_BN_BUFFERS)


class _PackTable:
    """Descriptor table for svk_pack_params: f32 master (flat) -> packed buffer (flat, dtype)."""

    def __init__(self, dtype):
        self.dtype = dtype
        self.rows = []
        self.trows = []          # transposed 2-D packs (svk_pack_transpose)
        self.total = 0           # packed buffer size
        self.gtotal = 0          # linear index space of the generic gather launch
        self.views = []

    def add(self, src, shape, strides, lims=None, view=None):
        n = [1] * (4 - len(shape)) + list(shape)
        s = [0] * (4 - len(strides)) + list(strides)
        lim = [1] * (4 - len(shape)) + list(lims if lims is not None else shape)
        numel = int(np.prod(shape))
        off = self.total
        if PACK_TRANSPOSE and len(shape) == 2 and tuple(strides) == (1, shape[0]) and lims is None:
            self.trows.append((src, off, shape[0], shape[1]))      # [K, N] view of a row-major [N, K] master
        else:
            self.rows.append((src, off, n, s, lim, self.gtotal))
            self.gtotal += (numel + 7) // 8 * 8    # 8-aligned descriptor starts: svk_pack_params8
        self.total += (numel + 7) // 8 * 8      # keep every packed tensor 16-byte aligned
        self.views.append((off, tuple(view or shape)))
        return len(self.views) - 1

    def finalize(self, device):
        arr = np.zeros(len(self.rows), dtype=_DESC)
        for i, (src, dst, n, s, lim, start) in enumerate(self.rows):
            arr[i] = (src, dst, n, s, lim, start)
        raw = torch.from_numpy(arr.view(np.uint8).copy())
        self.desc = raw.to(device)
        tiles = [(src, dst, K, N, n0, k0) for src, dst, K, N in self.trows
                 for n0 in range(0, N, 64) for k0 in range(0, K, 64)]
        self.ntiles = len(tiles)
        tarr = np.array(tiles, dtype=_TILE) if tiles else np.zeros(1, dtype=_TILE)
        self.tiles = torch.from_numpy(tarr.view(np.uint8).copy()).to(device)
        self.buf = torch.zeros(max(self.total, 8), device=device, dtype=self.dtype)
        self.tensors = [self.buf[o:o + int(np.prod(sh))].view(sh) for o, sh in self.views]

    def run(self, master, dst=None):
        out = self.buf if dst is None else dst
        if self.rows:
            if PACK_PARAMS8:
                ops.pack_params8(self.desc, len(self.rows), self.gtotal, master, out)
            else:
                ops.pack_params(self.desc, len(self.rows), self.gtotal, master, out)
        if self.ntiles:
            ops.pack_transpose(self.tiles, self.ntiles, master, out)


def _t(w):
    """Frozen weight -> transposed contiguous copy (one-time packing)."""
    return w.detach().t().contiguous()


class EVPTrainStep:
    """One optimizer step per call over a batch of frames; owns the flat parameter/gradient/momentum
    buffers of the trainable parameters.  ``process_group``: torch.distributed group for DDP
    (gradient all-reduce, BN buffer broadcast from rank 0); None = single process."""

    def __init__(self, model, lr=5e-4, momentum=0.9, dampening=0.0, weight_decay=1e-5, nesterov=False,
                 dtype=torch.bfloat16, drop=True, seed=0, process_group=None, world_size=1, grad_comm="f32"):
        if grad_comm not in ("f32", "bf16"):
            raise SvkError(f"EVPTrainStep: grad_comm must be 'f32' or 'bf16', got {grad_comm!r}")
        self.grad_comm = grad_comm
        self._comm = {}
        self.model = model
        self.dt = dtype
        self.hp = dict(lr=lr, momentum=momentum, dampening=dampening, weight_decay=weight_decay, nesterov=nesterov)
        self.drop = drop
        self.seed = seed
        self.group = process_group
        self.world = world_size
        self._bn_flat = None
        self.keep_saved, self.last_saved = False, None
        self.steps = 0
        dev = next(model.parameters()).device
        if dev.type != "cuda":
            raise SvkError("EVPTrainStep: model must be on a GPU (there is no CPU path)")
        self.dev = dev
        model.train()
        self.depths = list(model.depths)
        self.dims = list(model.embed_dims)
        self._setup_flat()
        self._setup_frozen()
        self._setup_packs()
        self.counter = torch.zeros(1, device=self.dev, dtype=torch.int64)   # device step count (mask RNG)
        self._mask_cache = {}
        self.graph = self.graph_rest = self.graph_opt = None
        self._pending = None

    # ---- parameter storage ------------------------------------------------------------------
    BIND_GRADS = True        # .grad of each trainable parameter = a view into the flat gradient

    def _setup_flat(self):
        tr = []
        for n, p in self.model.named_parameters():
            if self.BIND_GRADS:
                p.requires_grad_(is_trainable(n))
            elif p.requires_grad != is_trainable(n):
                raise SvkError(
                    "MixVisionTransformerEVP train mode on the svk kernels trains the reference's parameter set "
                    "(train_evp.py:379-382: names containing head / prompt / flow_encoder / cross_attn_s3 / "
                    f"cross_attn_s4, everything else frozen); parameter {n!r} has requires_grad={p.requires_grad}")
            if is_trainable(n):
                tr.append((n, p))
        # every tensor starts 16-byte aligned (offsets rounded up to 4 floats): the f32 biases are read by the
        # GEMM epilogues with 16-byte loads, and an unaligned one sent the GEMM to the legacy kernel; the gaps
        # stay zero (zero gradient, zero momentum, SGD keeps them at 0)
        self.off = {}
        o = 0
        align = 4 if os.environ.get("SVK_FLAT_ALIGN", "1") == "1" else 1
        for n, p in tr:
            self.off[n] = o
            o += (p.numel() + align - 1) // align * align
        total = o
        self.flat = torch.zeros(total, device=self.dev, dtype=torch.float32)
        self.grad = torch.zeros(total, device=self.dev, dtype=torch.float32)
        self.mom = torch.zeros(total, device=self.dev, dtype=torch.float32)
        with torch.no_grad():
            for n, p in tr:
                o, k = self.off[n], p.numel()
                self.flat[o:o + k].copy_(p.detach().reshape(-1))
                p.data = self.flat[o:o + k].view_as(p)
                if self.BIND_GRADS:
                    p.grad = self.grad[o:o + k].view_as(p)
        self.params = dict(tr)
        self.n_trainable = sum(p.numel() for _, p in tr)
        # the head's parameters lead the flat buffer (model construction order): its gradient bucket
        heads = [n for n, _ in tr if n.startswith("head.")]
        self.head_end = max((self.off[n] + self.params[n].numel() for n in heads), default=0)
        if any(not n.startswith("head.") and self.off[n] < self.head_end for n, _ in tr):
            self.head_end = 0                      # not a prefix: one bucket

    def P(self, name):
        """f32 master view of a trainable parameter."""
        return self.params[name]

    def G(self, name):
        """f32 gradient view of a trainable parameter (into the flat gradient buffer)."""
        p = self.params[name]
        o = self.off[name]
        return self.grad[o:o + p.numel()].view_as(p)

    # ---- packs --------------------------------------------------------------------------------
    def _setup_packs(self):
        dt = self.dt
        tab, tab32, un = _PackTable(dt), _PackTable(torch.float32), _PackTable(torch.float32)
        self.pk, self.pk32 = {}, {}
        conv_scratch = 0
        self.conv_grad = {}

        def lin(name, transposed=True):
            N, K = self.params[name].shape[:2]
            o = self.off[name]
            self.pk[name] = tab.add(o, (N, K), (K, 1))
            if transposed:
                self.pk[name + ".T"] = tab.add(o, (K, N), (1, K))

        def conv(name, dgrad, pad_in=False):
            nonlocal conv_scratch
            co, ci, k, _ = self.params[name].shape
            o = self.off[name]
            cp = pad_channels(ci) if pad_in else ci
            self.pk[name] = tab.add(o, (co, k, k, cp), (ci * k * k, k, 1, k * k), (co, k, k, ci), view=(co, k * k * cp))
            if dgrad:
                # (ci, k, k, co) = the 2-D transpose of the master's [co][ci * k * k] rows: the tiled transpose
                # kernel instead of the strided gather (round 6)
                if PACK_D_TRANSPOSE:
                    self.pk[name + ".D"] = tab.add(o, (ci * k * k, co), (1, ci * k * k), view=(ci, k * k * co))
                else:
                    self.pk[name + ".D"] = tab.add(o, (ci, k, k, co), (k * k, k, 1, ci * k * k), view=(ci, k * k * co))
                self.pk[name + ".C"] = tab.add(o, (k, k, ci, co), (k, 1, k * k, ci * k * k), view=(k * k * ci, co))
            # weight-gradient scratch in the packed layout, unpacked into the flat grad after backward
            n = co * k * k * cp
            self.conv_grad[name] = (conv_scratch, (co, k * k * cp))
            un_rows.append((conv_scratch, name, co, ci, k, cp))
            conv_scratch += (n + 7) // 8 * 8

        un_rows = []
        pg = "prompt_generator"
        for s in range(4):
            conv(f"{pg}.handcrafted_generator{s + 1}.proj.weight", dgrad=s > 0, pad_in=s == 0)
            lin(f"{pg}.embedding_generator{s + 1}.weight")
            lin(f"{pg}.shared_mlp{s + 1}.weight")
            for i in range(self.depths[s]):
                lin(f"{pg}.lightweight_mlp{s + 1}_{i}.0.weight")
        for i in range(1, 5):
            conv(f"flow_encoder.conv{i}.weight", dgrad=i > 1, pad_in=i == 1)
        for s in (3, 4):
            nm = f"cross_attn_s{s}.cross_attn.in_proj_weight"
            E = self.params[nm].shape[1]
            o = self.off[nm]
            self.pk[nm] = tab.add(o, (3 * E, E), (E, 1))
            self.pk[nm + ".qT"] = tab.add(o, (E, E), (1, E))
            self.pk[nm + ".kvT"] = tab.add(o + E * E, (E, 2 * E), (1, E))
            lin(f"cross_attn_s{s}.cross_attn.out_proj.weight")
        for i in range(1, 5):
            lin(f"head.linear_c{i}.proj.weight")
        nm = "head.linear_fuse.conv.weight"
        E, K = self.params[nm].shape[:2]
        self.pk[nm] = tab.add(self.off[nm], (E, K), (K, 1))
        self.pk[nm + ".T"] = tab.add(self.off[nm], (K, E), (1, K))
        for h in ("fc", "fc_ant"):
            for j in (0, 2):
                nm = f"head.{h}.{j}.weight"
                N, K = self.params[nm].shape
                self.pk32[nm + ".T"] = tab32.add(self.off[nm], (K, N), (1, K))
        # packed conv grads -> flat grad ([co][k][k][cp] -> [co][ci][k][k])
        for sc, name, co, ci, k, cp in un_rows:
            un.add(sc, (co, ci, k, k), (k * k * cp, 1, k * cp, cp))
        for t in (tab, tab32, un):
            t.finalize(self.dev)
        self.tab, self.tab32, self.untab = tab, tab32, un
        self.conv_scratch = torch.zeros(max(conv_scratch, 8), device=self.dev, dtype=torch.float32)
        # the unpack table writes into the flat gradient at each conv weight's offset
        for i, (sc, name, co, ci, k, cp) in enumerate(un_rows):
            self.untab.rows[i] = (sc, self.off[name], *self.untab.rows[i][2:5], self.untab.rows[i][5])
        arr = np.zeros(len(self.untab.rows), dtype=_DESC)
        for i, r in enumerate(self.untab.rows):
            arr[i] = r
        self.untab.desc = torch.from_numpy(arr.view(np.uint8).copy()).to(self.dev)
        self._refresh_packs()

    def _refresh_packs(self):
        self.tab.run(self.flat)
        self.tab32.run(self.flat)

    def W(self, key):
        return self.tab.tensors[self.pk[key]]

    def W32T(self, key):
        return self.tab32.tensors[self.pk32[key]]

    def CG(self, name):
        o, shape = self.conv_grad[name]
        return self.conv_scratch[o:o + shape[0] * shape[1]].view(shape)

    def _setup_frozen(self):
        """One-time packs of the frozen backbone (forward and adjoint layouts)."""
        m, dt = self.model, self.dt
        self.fz = []
        with torch.no_grad():
            for s in range(4):
                pe = getattr(m, f"patch_embed{s + 1}")
                w = pe.proj.weight.detach()
                co, ci, k, _ = w.shape
                st = dict(k=k, stride=pe.stride, pad=k // 2)
                st["w"] = conv_w(w, dt, pad_channels(ci))
                if s == 0 and ops.stem_s2d_ok(dt, ci, k, pe.stride):
                    st["w_s2d"] = conv_w_s2d(w, dt, pe.stride)
                st["wd"] = w.permute(1, 2, 3, 0).reshape(ci, k * k * co).to(dt).contiguous() if s > 0 else None
                # col2im adjoint layout [(ky, kx, ci), co]
                st["wc"] = w.permute(2, 3, 1, 0).reshape(k * k * ci, co).to(dt).contiguous() if s > 0 else None
                st["b"] = pe.proj.bias.detach().float().contiguous()
                st["g"], st["beta"] = pe.norm.weight.detach().float().contiguous(), pe.norm.bias.detach().float().contiguous()
                norm = getattr(m, f"norm{s + 1}")
                st["ng"], st["nb"] = norm.weight.detach().float().contiguous(), norm.bias.detach().float().contiguous()
                blocks = []
                for blk in getattr(m, f"block{s + 1}"):
                    a, f = blk.attn, blk.mlp
                    C = a.dim
                    b = dict(heads=a.num_heads, scale=a.scale, sr=a.sr_ratio,
                             g1=blk.norm1.weight.detach().float().contiguous(),
                             b1=blk.norm1.bias.detach().float().contiguous(),
                             g2=blk.norm2.weight.detach().float().contiguous(),
                             b2=blk.norm2.bias.detach().float().contiguous(),
                             wq=a.q.weight.detach().to(dt).contiguous(), bq=a.q.bias.detach().float().contiguous(),
                             wqT=_t(a.q.weight).to(dt), wkv=a.kv.weight.detach().to(dt).contiguous(),
                             bkv=a.kv.bias.detach().float().contiguous(), wkvT=_t(a.kv.weight).to(dt),
                             wp=a.proj.weight.detach().to(dt).contiguous(),
                             bp=a.proj.bias.detach().float().contiguous(), wpT=_t(a.proj.weight).to(dt),
                             w1=f.fc1.weight.detach().to(dt).contiguous(), bf1=f.fc1.bias.detach().float().contiguous(),
                             w1T=_t(f.fc1.weight).to(dt), w2=f.fc2.weight.detach().to(dt).contiguous(),
                             bf2=f.fc2.bias.detach().float().contiguous(), w2T=_t(f.fc2.weight).to(dt))
                    dw = f.dwconv.dwconv
                    hid = dw.weight.shape[0]
                    taps = dw.weight.detach().float().reshape(hid, 9).t().contiguous()
                    b["taps"], b["dwb"] = taps, dw.bias.detach().float().contiguous()
                    b["taps_flip"] = taps.flip(0).contiguous()
                    b["zero"] = torch.zeros(hid, device=self.dev, dtype=torch.float32)
                    if a.sr_ratio > 1:
                        r = a.sr_ratio
                        wsr = a.sr.weight.detach()
                        b["wsr"] = conv_w(wsr, dt)
                        b["bsr"] = a.sr.bias.detach().float().contiguous()
                        b["wsrD"] = wsr.permute(2, 3, 1, 0).reshape(r * r * C, C).to(dt).contiguous()
                        b["gn"] = a.norm.weight.detach().float().contiguous()
                        b["bn"] = a.norm.bias.detach().float().contiguous()
                    blocks.append(b)
                st["blocks"] = blocks
                self.fz.append(st)

    # ---- masks ----------------------------------------------------------------------------------
    def make_masks(self, B):
        """Device DropPath / Dropout2d masks for this step (values 0 or 1/keep)."""
        dpr = torch.linspace(0, DROP_PATH_RATE, sum(self.depths)).tolist()
        blocks, cur = [], 0
        base = (self.seed * 1000003) & 0x7FFFFFFF      # the step enters through the device counter
        # constant per (B, schedule): the ones rows and the per-mask keep / seed tables, built once (eagerly,
        # before any capture) so a replayed step holds no fill or copy nodes for them
        key = ("mask_tables", B, self.drop, base)
        if key not in self._mask_cache:
            keeps, seeds = [], []
            for k in range(sum(self.depths)):
                if self.drop and dpr[k] > 0:
                    for j in range(2):
                        keeps.append(1.0 - dpr[k])
                        seeds.append((base + 2 * k + j) & 0xFFFFFFFF)
            kt = torch.tensor(keeps, dtype=torch.float32).to(self.dev)
            st_ = torch.tensor([v - (1 << 32) if v >= 1 << 31 else v for v in seeds], dtype=torch.int32).to(self.dev)
            self._mask_cache[key] = (torch.ones(B, device=self.dev, dtype=torch.float32), kt, st_)
        ones, kt, st_ = self._mask_cache[key]
        # every block's two DropPath masks in one launch (rows in block order), bit-identical to keep_mask
        allm = ops.keep_mask_multi(B, kt, st_, self.counter) if kt.numel() and TRAIN_MASK_MULTI else None
        mi = 0
        for s, d in enumerate(self.depths):
            st = []
            for i in range(d):
                r = dpr[cur + i]
                if self.drop and r > 0 and allm is not None:
                    st.append((allm[mi], allm[mi + 1]))
                    mi += 2
                elif self.drop and r > 0:
                    st.append(tuple(ops.keep_mask(B, 1.0 - r, base + 2 * (cur + i) + j, self.dev, self.counter)
                                    for j in range(2)))
                else:
                    st.append((ones, ones))
            blocks.append(st)
            cur += d
        if self.drop:
            d2 = ops.keep_mask(B * 2048, 1.0 - HEAD_DROPOUT, base + 99991, self.dev, self.counter).view(B, 2048)
        else:
            d2 = torch.ones(B, 2048, device=self.dev, dtype=torch.float32)
        return {"blocks": blocks, "dropout2d": d2}

    # ---- forward ----------------------------------------------------------------------------------
    def _forward(self, x, y, flow, masks):
        dt, pg = self.dt, "prompt_generator"
        B = x.numel() // (3 * 224 * 224)
        sv = {"B": B}
        # handcrafted prompt cascade (trainable; mix_transformer_evp.py:718-747)
        prev = ops.gauss5x5_reflect(y.reshape(B, 3, 224, 224).float(), dt, cpad=8)
        hc = []
        for s in range(4):
            nm = f"{pg}.handcrafted_generator{s + 1}"
            k, st = (7, 4) if s == 0 else (3, 2)
            z = ops.conv2d_nhwc(prev, self.W(nm + ".proj.weight"), k, st, k // 2, bias=self.P(nm + ".proj.bias"))
            _, OH, OW, C = z.shape
            h = ops.layernorm(z.view(B, OH * OW, C), self.P(nm + ".norm.weight"), self.P(nm + ".norm.bias"), LN_EPS)
            hc.append(dict(inp=prev, z=z, h=h, k=k, st=st, H=OH, W=OW, C=C))
            prev = h.view(B, OH, OW, C)
        sv["hc"] = hc
        # backbone with prompts (frozen weights; mix_transformer_evp.py:352-416)
        x4 = x.reshape(B, 3, 224, 224).float()
        cur = None if "w_s2d" in self.fz[0] else ops.nchw_to_nhwc(x4, dt, cpad=8)
        stages = []
        for s in range(4):
            fz = self.fz[s]
            if cur is None:     # frozen stem over space-to-depth blocks (no data / weight gradient needed)
                z = ops.conv2d_stem_s2d(x4, fz["w_s2d"], fz["k"], fz["stride"], fz["pad"], bias=fz["b"])
                cur = x4.permute(0, 2, 3, 1)         # shape-only stand-in for in_hw (read for s > 0 only)
            else:
                z = ops.conv2d_nhwc(cur, fz["w"], fz["k"], fz["stride"], fz["pad"], bias=fz["b"])
            _, H, W, C = z.shape
            N = H * W
            t = ops.layernorm(z.view(B, N, C), fz["g"], fz["beta"], LN_EPS)
            eg = f"{pg}.embedding_generator{s + 1}"
            summed = ops.gemm(t, self.W(eg + ".weight"), self.P(eg + ".bias"), residual=hc[s]["h"])
            st = dict(in_hw=(cur.shape[1], cur.shape[2], cur.shape[3]), z=z, t=t, summed=summed, H=H, W=W, C=C, N=N,
                      blocks=[])
            x_ = t
            sh = f"{pg}.shared_mlp{s + 1}"
            for i, b in enumerate(fz["blocks"]):
                lw = f"{pg}.lightweight_mlp{s + 1}_{i}.0"
                fpre = ops.gemm(summed, self.W(lw + ".weight"), self.P(lw + ".bias"))
                f = ops.gemm(summed, self.W(lw + ".weight"), self.P(lw + ".bias"), act="gelu")
                xp = ops.gemm(f, self.W(sh + ".weight"), self.P(sh + ".bias"), residual=x_)
                ma, mm = masks["blocks"][s][i]
                sb = self._block_fwd(xp, b, B, H, W, C, ma, mm)
                sb.update(fpre=fpre, f=f, xp=xp, ma=ma, mm=mm)
                st["blocks"].append(sb)
                x_ = sb["out"]
            st["last"] = x_
            c = ops.layernorm(x_, fz["ng"], fz["nb"], BLOCK_EPS)
            st["c"] = c
            stages.append(st)
            cur = c.view(B, H, W, C)
        sv["stages"] = stages
        # flow encoder, BN in train mode
        fl = []
        prev = ops.nchw_to_nhwc(flow.reshape(B, 2, 224, 224).float(), dt, cpad=8)
        for i, (k, st_, pad) in enumerate(((7, 4, 3), (3, 2, 1), (3, 2, 1), (3, 2, 1)), start=1):
            nm = f"flow_encoder.conv{i}"
            z = ops.conv2d_nhwc(prev, self.W(nm + ".weight"), k, st_, pad, bias=self.P(nm + ".bias"))
            Cz = z.shape[-1]
            s1, s2 = ops.colstats_set(z.view(-1, Cz))          # written, not accumulated: no zero-fills
            bn = f"flow_encoder.bn{i}"
            yb = ops.bn_apply(z, s1, s2, self.P(bn + ".weight"), self.P(bn + ".bias"), BN_EPS, act="relu")
            fl.append(dict(inp=prev, z=z, y=yb, s1=s1, s2=s2, k=k, st=st_, pad=pad))
            prev = yb
        sv["flow"] = fl
        # motion-guided cross attention on c3 / c4
        ca = {}
        for s in (3, 4):
            c = stages[s - 1]["c"]
            f = fl[s - 1]["y"]
            f = f.view(B, -1, f.shape[-1])
            ca[s] = self._cross_fwd(s, c, f)
        sv["ca"] = ca
        # head, train mode
        sv["head"] = hd = self._head_fwd(B, [stages[0]["c"], stages[1]["c"], ca[3]["out"], ca[4]["out"]],
                                         [(st["H"], st["W"]) for st in stages], masks["dropout2d"])
        return sv, hd["logits"], hd["ant"]

    def _block_fwd(self, xp, b, B, H, W, C, ma, mm):
        N = H * W
        xn1 = ops.layernorm(xp, b["g1"], b["b1"], BLOCK_EPS)
        q = ops.gemm(xn1, b["wq"], b["bq"])
        sv = {}
        if b["sr"] > 1:
            r = b["sr"]
            xs_pre = ops.conv2d_nhwc(xn1.view(B, H, W, C), b["wsr"], r, r, 0, bias=b["bsr"]).view(B, -1, C)
            xs = ops.layernorm(xs_pre, b["gn"], b["bn"], LN_EPS)
            sv["xs_pre"] = xs_pre
        else:
            xs = xn1
        kv = ops.gemm(xs, b["wkv"], b["bkv"])
        o = ops.attention(q, kv[:, :, :C], kv[:, :, C:], b["heads"], b["scale"])
        x1 = ops.gemm(o, b["wp"], b["bp"], residual=xp, row_scale=ma, rows_per=N)
        xn2 = ops.layernorm(x1, b["g2"], b["b2"], BLOCK_EPS)
        hid = b["w1"].shape[0]
        u = torch.empty(B, H, W, hid, device=self.dev, dtype=self.dt)
        if TRAIN_FC1_DWCONV and self.dt in ops.H16 and C in TRAIN_FC1_DWCONV_C and hid % 64 == 0:
            # fc1 -> DWConv (+ pre-activation for the GELU backward) -> GELU in one kernel: the frozen fc1's
            # output is never needed by the backward, so it stays on chip (Mlp.forward :60-63)
            g = ops.mixffn_fc1_dwconv(xn2.view(B, H, W, C), b["w1"], b["bf1"], b["taps"], b["dwb"], act="gelu",
                                      pre_out=u)
        else:
            h = ops.gemm(xn2, b["w1"], b["bf1"])
            pk = self._dwfc_fwd_pack(b, H, W, C) if TRAIN_DWFC_FWD and self.dt in ops.H16 else None
            if pk is not None:
                # stages 3-4 (round 6): DWConv + GELU + fc2 (+ DropPath scale, residual) in one matrix-core kernel
                # that also stores the pre-activation u for the GELU backward — the GELU map never reaches HBM
                out = ops.mixffn_dw_fc2(h.view(B, H, W, hid), b["taps"], b["dwb"], b["w2"], b["bf2"], residual=x1,
                                        packed=pk, pre_out=u, row_scale=mm, rows_per=N)
                sv.update(q=q, kv=kv, o=o, x1=x1, u=u, out=out)
                return sv
            g = ops.dwconv3x3(h.view(B, H, W, hid), b["taps"], b["dwb"], act="gelu", pre_out=u)
        out = ops.gemm(g.view(B, N, hid), b["w2"], b["bf2"], residual=x1, row_scale=mm, rows_per=N)
        sv.update(q=q, kv=kv, o=o, x1=x1, u=u, out=out)
        return sv

    def _cross_fwd(self, s, c, f):
        p = f"cross_attn_s{s}"
        E = c.shape[-1]
        wi = self.W(p + ".cross_attn.in_proj_weight")
        bi = self.P(p + ".cross_attn.in_proj_bias")
        q = ops.gemm(c, wi[:E], bi[:E])
        kv = ops.gemm(f, wi[E:], bi[E:])
        heads = 8
        o = ops.attention(q, kv[:, :, :E], kv[:, :, E:], heads, (E // heads) ** -0.5)
        a = ops.gemm(o, self.W(p + ".cross_attn.out_proj.weight"), self.P(p + ".cross_attn.out_proj.bias"), residual=c)
        out = ops.layernorm(a, self.P(p + ".norm.weight"), self.P(p + ".norm.bias"), LN_EPS)
        return dict(c=c, f=f, q=q, kv=kv, o=o, a=a, out=out, E=E, heads=heads)

    def _head_fwd(self, B, toks, hw, d2mask):
        H4, W4 = hw[3]
        R = H4 * W4
        Ed = 2048
        E = torch.empty(B * R, 4 * Ed, device=self.dev, dtype=self.dt)
        rs = []
        for j, lvl in enumerate((3, 2, 1, 0)):             # torch.cat([_c4, _c3, _c2, _c1]) (segformer_head.py:158)
            t = toks[lvl]
            H, W = hw[lvl]
            r = t if (H, W) == (H4, W4) else ops.resize_bilinear(t, H, W, H4, W4)
            r = r.reshape(B * R, -1)
            nm = f"head.linear_c{lvl + 1}.proj"
            ops.gemm(r, self.W(nm + ".weight"), self.P(nm + ".bias"), out=E[:, j * Ed:(j + 1) * Ed])
            rs.append((lvl, r, H, W))
        Z = ops.gemm(E, self.W("head.linear_fuse.conv.weight"))
        s1, s2 = ops.colstats_set(Z)
        bn = "head.linear_fuse.bn"
        Yb = ops.bn_apply(Z, s1, s2, self.P(bn + ".weight"), self.P(bn + ".bias"), BN_EPS, act="relu")
        feat = ops.mul_f32(ops.mean_rows(Yb, R), d2mask)
        outs, hs = [], []
        for h in ("fc", "fc_ant"):
            h1 = ops.gemm(feat, self.P(f"head.{h}.0.weight"), self.P(f"head.{h}.0.bias"), act="relu")
            outs.append(ops.gemm(h1, self.P(f"head.{h}.2.weight"), self.P(f"head.{h}.2.bias")))
            hs.append(h1)
        return dict(E=E, rs=rs, Z=Z, s1=s1, s2=s2, feat=feat, hs=hs, logits=outs[0], ant=outs[1], R=R, d2=d2mask)

    # ---- backward ---------------------------------------------------------------------------------
    def _wg(self, dy, x, name, bias_name=None):
        """Linear weight/bias gradients: dW += dy^T x; db += colsum(dy) (one fused kernel)."""
        ops.gemm_wgrad(dy.reshape(-1, dy.shape[-1]), x.reshape(-1, x.shape[-1]), self.G(name),
                       None if bias_name is None else self.G(bias_name))

    def _backward(self, sv, dlogits, dant):
        self._backward_rest(sv, self._backward_head(sv, dlogits, dant))

    def _backward_head(self, sv, dlogits, dant):
        """SegFormerHead backward: after it every head.* gradient (the first, 85 % of the flat gradient
        buffer) is final, so DDP can all-reduce that bucket while the backbone backward runs."""
        dt, B = self.dt, sv["B"]
        hd = sv["head"]
        # fc / fc_ant (f32)
        dfeat = None
        for h, dl, h1 in (("fc", dlogits, hd["hs"][0]), ("fc_ant", dant, hd["hs"][1])):
            self._wg(dl, h1, f"head.{h}.2.weight", f"head.{h}.2.bias")
            dh = ops.gemm(dl, self.W32T(f"head.{h}.2.weight.T"), dact="relu", dact_src=h1)
            self._wg(dh, hd["feat"], f"head.{h}.0.weight", f"head.{h}.0.bias")
            dfeat = ops.gemm(dh, self.W32T(f"head.{h}.0.weight.T"), residual=dfeat)
        # Dropout2d + average pool + BN(train) + ReLU
        R = hd["R"]
        dY = ops.bcast_rows(dfeat, R, dt, scale=1.0 / R, mask=hd["d2"])
        bn = "head.linear_fuse.bn"
        dZ = ops.bn_bwd(hd["Z"], dY, hd["s1"], hd["s2"], self.P(bn + ".weight"), self.P(bn + ".bias"), BN_EPS,
                        self.G(bn + ".weight"), self.G(bn + ".bias"), relu=True)
        ops.gemm_wgrad(dZ, hd["E"], self.G("head.linear_fuse.conv.weight").view(2048, -1))
        dE = ops.gemm(dZ, self.W("head.linear_fuse.conv.weight.T"))
        dtok = [None] * 4
        for j, (lvl, r, H, W) in enumerate(hd["rs"]):
            dEj = dE[:, j * 2048:(j + 1) * 2048]
            nm = f"head.linear_c{lvl + 1}.proj"
            self._wg(dEj, r, nm + ".weight", nm + ".bias")
            dr = ops.gemm(dEj, self.W(nm + ".weight.T"))
            if (H * W) == R:
                dtok[lvl] = dr.view(B, R, -1)
            else:
                acc = torch.zeros(B, H * W, dr.shape[-1], device=self.dev, dtype=torch.float32)
                ops.resize_bilinear_bwd(dr.view(B, R, -1), H, W, 7, 7, acc)
                dtok[lvl] = ops.cast(acc, dt)
        return dtok

    def _backward_rest(self, sv, dtok):
        dt, B, pg = self.dt, sv["B"], "prompt_generator"
        stages = sv["stages"]
        # cross attention (s4, s3) -> grads of backbone c3/c4 and of the flow features
        dflow = {}
        for s in (4, 3):
            dtok[s - 1], dflow[s] = self._cross_bwd(s, sv["ca"][s], dtok[s - 1])
        self._flow_bwd(sv["flow"], dflow, B)
        # backbone, stage 4 -> 1
        dhc = [None] * 4
        dnext = None
        for s in range(3, -1, -1):
            st, fz = stages[s], self.fz[s]
            dc = dtok[s].reshape(B, st["N"], st["C"])
            if dnext is not None:
                dc = dnext
            d = ops.layernorm_bwd(st["last"], dc, fz["ng"], BLOCK_EPS)
            dsum = None
            sh = f"{pg}.shared_mlp{s + 1}"
            for i in range(len(fz["blocks"]) - 1, -1, -1):
                b, sb = fz["blocks"][i], st["blocks"][i]
                d = self._block_bwd(d, b, sb, B, st["H"], st["W"], st["C"])
                # prompt: xp = x + shared(GELU(lw_i(summed)))
                lw = f"{pg}.lightweight_mlp{s + 1}_{i}.0"
                self._wg(d, sb["f"], sh + ".weight", sh + ".bias")
                dfp = ops.gemm(d, self.W(sh + ".weight.T"), dact="gelu", dact_src=sb["fpre"])
                self._wg(dfp, st["summed"], lw + ".weight", lw + ".bias")
                dsum = ops.gemm(dfp, self.W(lw + ".weight.T"), residual=dsum, out=dsum)
            eg = f"{pg}.embedding_generator{s + 1}"
            self._wg(dsum, st["t"], eg + ".weight", eg + ".bias")
            d = ops.gemm(dsum, self.W(eg + ".weight.T"), residual=d, out=d)
            dhc[s] = dsum
            if s > 0:
                # frozen patch embed: LN backward then conv data gradient, added to the previous stage's grad
                dz = ops.layernorm_bwd(st["z"].view(B, st["N"], st["C"]), d, fz["g"], LN_EPS)
                Hp, Wp, Cp = st["in_hw"]
                prev = dtok[s - 1].reshape(B, Hp, Wp, Cp).contiguous()
                dzm = dz.view(B, st["H"], st["W"], st["C"])
                if TRAIN_COL2IM and self.dt in ops.H16 and Cp % 8 == 0:
                    dnext = ops.conv2d_dgrad_col2im(dzm, fz["wc"], Hp, Wp, Cp, fz["k"], fz["stride"], fz["pad"],
                                                    residual=prev).view(B, Hp * Wp, Cp)
                else:
                    dnext = ops.conv2d_dgrad(dzm, fz["wd"], Hp, Wp, Cp, fz["k"], fz["stride"], fz["pad"],
                                             residual=prev).view(B, Hp * Wp, Cp)
        # handcrafted cascade backward (trainable convs + LNs)
        dh = dhc[3]
        for s in range(3, -1, -1):
            h = sv["hc"][s]
            nm = f"{pg}.handcrafted_generator{s + 1}"
            dz = ops.layernorm_bwd(h["z"].view(B, h["H"] * h["W"], h["C"]), dh.view(B, h["H"] * h["W"], h["C"]),
                                   self.P(nm + ".norm.weight"), LN_EPS, dgamma=self.G(nm + ".norm.weight"),
                                   dbeta=self.G(nm + ".norm.bias"))
            dzm = dz.view(B, h["H"], h["W"], h["C"])
            ops.conv2d_wgrad(h["inp"], dzm, h["k"], h["st"], h["k"] // 2, self.CG(nm + ".proj.weight"),
                             self.G(nm + ".proj.bias"))
            if s > 0:
                pin = h["inp"]
                dg = (ops.conv2d_dgrad_col2im if TRAIN_COL2IM and self.dt in ops.H16 and pin.shape[3] % 8 == 0
                      else ops.conv2d_dgrad)
                dh = dg(dzm, self.W(nm + ".proj.weight." + ("C" if dg is ops.conv2d_dgrad_col2im else "D")),
                        pin.shape[1], pin.shape[2], pin.shape[3], h["k"], h["st"], h["k"] // 2,
                        residual=dhc[s - 1].view(pin.shape).contiguous())

    def _dwfc_fwd_pack(self, b, H, W, C):
        """The packed operands of the fused training-forward DWConv + GELU + fc2 (forward taps, the DWConv bias,
        W2) for this block's map, or None where the matrix-core dw_fc2 has no training form (14 x 14 / 7 x 7 only;
        cached in the block's parameter dict)."""
        key = ("dwfc_fwd", H, W)
        if key not in b:
            pk = None
            if H == W and W in (7, 14) and ops.mixffn_dw_fc2_supported(self.dt, W, C, b["w2"].shape[1]):
                pk = ops.mixffn_dw_fc2_pack(b["taps"], b["dwb"], b["w2"], W)
            b[key] = pk
        return b[key]

    def _dwfc_bwd_pack(self, b, H, W, C):
        """The packed operands of the fused DWConv + fc1 data gradient for this block's map, or None where
        the matrix-core dw_fc2 has no form for it (cached in the block's parameter dict)."""
        key = ("dwfc_bwd", H, W)
        if key not in b:
            pk = None
            if H == W and ops.mixffn_dw_fc2_supported(self.dt, W, C, b["w1T"].shape[1]):
                pk = ops.mixffn_dw_fc2_pack(b["taps_flip"], b["zero"], b["w1T"], W)
            if pk is not None and W == 28:
                pk = None                                     # (no identity-activation form at 28 x 28)
            b[key] = pk
            b["zeroC"] = torch.zeros(C, device=self.dev, dtype=torch.float32)
        return b[key]

    def _block_bwd(self, d, b, sb, B, H, W, C):
        """Data gradient through one frozen block (given d = dL/d out) -> dL/d xp."""
        N = H * W
        hid = sb["u"].shape[-1]
        du = ops.gemm(d, b["w2T"], row_scale=sb["mm"], rows_per=N, dact="gelu", dact_src=sb["u"].view(B, N, hid))
        pk = self._dwfc_bwd_pack(b, H, W, C) if TRAIN_DWFC_BWD and self.dt in ops.H16 else None
        if pk is not None:
            # dX = (dwconv3x3ᵀ dU) W1 in one kernel: the depthwise map never reaches HBM
            dxn2 = ops.mixffn_dw_fc2(du.view(B, H, W, hid), b["taps_flip"], b["zero"], b["w1T"], b["zeroC"],
                                     packed=pk, act="none").view(B, N, C)
        else:
            dh = ops.dwconv3x3(du.view(B, H, W, hid), b["taps_flip"], b["zero"]).view(B, N, hid)
            dxn2 = ops.gemm(dh, b["w1T"])
        d1 = ops.layernorm_bwd(sb["x1"], dxn2, b["g2"], BLOCK_EPS, dres=d)
        do = ops.gemm(d1, b["wpT"], row_scale=sb["ma"], rows_per=N)
        kv = sb["kv"]
        Nk = kv.shape[1]
        dkv = torch.empty(B, Nk, 2 * C, device=self.dev, dtype=self.dt)
        dq, _, _ = ops.attention_bwd(sb["q"], kv[:, :, :C], kv[:, :, C:], sb["o"], do, b["heads"], b["scale"],
                                     dkv[:, :, :C], dkv[:, :, C:])
        dxs = ops.gemm(dkv, b["wkvT"])
        if b["sr"] > 1:
            r = b["sr"]
            dxs_pre = ops.layernorm_bwd(sb["xs_pre"], dxs, b["gn"], LN_EPS)
            dxn1 = ops.gemm(dq, b["wqT"])
            if TRAIN_UNPATCHIFY_SPLIT and self.dt in ops.H16:
                # sequence-reduction conv data gradient: the patch-row GEMM on the persistent kernel, then one
                # vectorised scatter-add into the pixel map (the fused scatter epilogue of the register-staged
                # GEMM ran at ~1 TB/s)
                pr = ops.gemm(dxs_pre.view(-1, C), b["wsrD"])
                ops.unpatchify(pr, B, H // r, W // r, r, C, dxn1.view(B, H, W, C), accumulate=True)
            else:
                ops.gemm_unpatchify(dxs_pre.view(-1, C), b["wsrD"], dxn1.view(B, H, W, C), r,
                                    residual=dxn1.view(B, H, W, C))
        else:
            dxn1 = ops.gemm(dq, b["wqT"], residual=dxs)
        return ops.layernorm_bwd(sb["xp"], dxn1, b["g1"], BLOCK_EPS, dres=d1)

    def _cross_bwd(self, s, ca, dout):
        p = f"cross_attn_s{s}"
        E, heads = ca["E"], ca["heads"]
        B = ca["c"].shape[0]
        da = ops.layernorm_bwd(ca["a"], dout.reshape(ca["a"].shape), self.P(p + ".norm.weight"), LN_EPS,
                               dgamma=self.G(p + ".norm.weight"), dbeta=self.G(p + ".norm.bias"))
        op = p + ".cross_attn.out_proj"
        self._wg(da, ca["o"], op + ".weight", op + ".bias")
        do = ops.gemm(da, self.W(op + ".weight.T"))
        kv = ca["kv"]
        Nk = kv.shape[1]
        dkv = torch.empty(B, Nk, 2 * E, device=self.dev, dtype=self.dt)
        dq, _, _ = ops.attention_bwd(ca["q"], kv[:, :, :E], kv[:, :, E:], ca["o"], do, heads, (E // heads) ** -0.5,
                                     dkv[:, :, :E], dkv[:, :, E:])
        ip = p + ".cross_attn.in_proj_weight"
        gW, gb = self.G(ip), self.G(p + ".cross_attn.in_proj_bias")
        ops.gemm_wgrad(dq.reshape(-1, E), ca["c"].reshape(-1, E), gW[:E], gb[:E])
        ops.gemm_wgrad(dkv.reshape(-1, 2 * E), ca["f"].reshape(-1, E), gW[E:], gb[E:])
        dc = ops.gemm(dq, self.W(ip + ".qT"), residual=da)
        df = ops.gemm(dkv, self.W(ip + ".kvT"))
        return dc, df

    def _flow_bwd(self, fl, dflow, B):
        dy = None
        for i in range(4, 0, -1):
            L = fl[i - 1]
            z = L["z"]
            if i == 4:
                dy = dflow[4].reshape(z.shape)
            bn = f"flow_encoder.bn{i}"
            dz = ops.bn_bwd(z, dy.reshape(z.shape).contiguous(), L["s1"], L["s2"], self.P(bn + ".weight"),
                            self.P(bn + ".bias"), BN_EPS, self.G(bn + ".weight"), self.G(bn + ".bias"), relu=True)
            nm = f"flow_encoder.conv{i}"
            ops.conv2d_wgrad(L["inp"], dz, L["k"], L["st"], L["pad"], self.CG(nm + ".weight"), self.G(nm + ".bias"))
            if i > 1:
                pin = L["inp"]
                res = dflow[3].reshape(pin.shape).contiguous() if i == 4 else None
                if TRAIN_COL2IM and self.dt in ops.H16 and pin.shape[3] % 8 == 0:
                    dy = ops.conv2d_dgrad_col2im(dz, self.W(nm + ".weight.C"), pin.shape[1], pin.shape[2],
                                                 pin.shape[3], L["k"], L["st"], L["pad"], residual=res)
                else:
                    dy = ops.conv2d_dgrad(dz, self.W(nm + ".weight.D"), pin.shape[1], pin.shape[2], pin.shape[3],
                                          L["k"], L["st"], L["pad"], residual=res)

    # ---- the step ---------------------------------------------------------------------------------
    def forward_backward(self, x, y, flow, labels, ant_targets, masks=None):
        """Zero grads, forward (train mode), loss, backward.  Returns (loss [2] f32 device tensor
        = (CE sum, SmoothL1 sum), logits, anticipation).  No collective runs in here (with DDP the
        caller syncs the BN buffers before and all-reduces the gradient buckets after, outside any
        captured graph: train_iteration / _replay)."""
        out = self.fb_head(x, y, flow, labels, ant_targets, masks)
        self.fb_rest()
        return out

    def fb_head(self, x, y, flow, labels, ant_targets, masks=None):
        """First part of forward_backward: zero grads, forward, loss, head backward (the head bucket of
        the gradient is final afterwards)."""
        B = x.numel() // (3 * 224 * 224)
        if masks is None:
            masks = self.make_masks(B)
        else:
            masks = {"blocks": [[(a.to(self.dev, torch.float32), b.to(self.dev, torch.float32)) for a, b in st]
                                for st in masks["blocks"]],
                     "dropout2d": masks["dropout2d"].to(self.dev, torch.float32).contiguous()}
        self.grad.zero_()
        self.conv_scratch.zero_()
        sv, logits, ant = self._forward(x, y, flow, masks)
        if self.keep_saved:                   # tests: the forward's saved tensors (BN sums, ReLU outputs)
            self.last_saved = sv
        loss, dl, da = ops.phase_loss(logits, ant, labels, ant_targets)
        self._pending = (sv, self._backward_head(sv, dl, da))
        return loss, logits, ant

    def fb_rest(self):
        """Second part: backbone / cross-attention / flow / prompt backward, conv-grad unpack, BN
        running statistics."""
        sv, dtok = self._pending
        self._pending = None
        self._backward_rest(sv, dtok)
        self.untab.run(self.conv_scratch, self.grad)   # packed conv weight grads -> flat grad (f32 gather)
        self._update_bn_running(sv)

    def _update_bn_running(self, sv):
        m = self.model
        mods = [(m.head.linear_fuse.bn, sv["head"]["s1"], sv["head"]["s2"], sv["head"]["Z"].shape[0])]
        for i, L in enumerate(sv["flow"], start=1):
            mods.append((getattr(m.flow_encoder, f"bn{i}"), L["s1"], L["s2"], L["z"].numel() // L["z"].shape[-1]))
        for bn, s1, s2, M in mods:
            ops.bn_update_running(s1, s2, M, bn.running_mean, bn.running_var, BN_MOMENTUM)
            bn.num_batches_tracked.add_(1)

    def _broadcast_buffers(self):
        """The five BatchNorms' running statistics from rank 0 as ONE collective: packed into a flat
        buffer, broadcast, unpacked (was ten separate broadcasts per step)."""
        import torch.distributed as dist
        m = self.model
        bufs = []
        for bn in [m.head.linear_fuse.bn] + [getattr(m.flow_encoder, f"bn{i}") for i in range(1, 5)]:
            bufs += [bn.running_mean, bn.running_var]
        flat = getattr(self, "_bn_flat", None)
        if flat is None:
            flat = self._bn_flat = torch.empty(sum(b.numel() for b in bufs), device=bufs[0].device,
                                               dtype=torch.float32)
        torch.cat([b.reshape(-1).float() for b in bufs], out=flat)
        dist.broadcast(flat, 0, group=self.group)
        off = 0
        for b in bufs:
            b.copy_(flat[off:off + b.numel()].view_as(b))
            off += b.numel()

    def _ddp(self):
        # a process group means DDP semantics at any world size (world 1 still runs the RCCL calls)
        return self.group is not None

    def sync_buffers(self):
        """DDP's broadcast_buffers: BN running statistics from rank 0, once per step, before the forward
        (eager, never inside a captured graph)."""
        if self._ddp():
            self._broadcast_buffers()

    def _grad_buckets(self):
        """Gradient all-reduce buckets, in the order backward finalises them: the head prefix of the flat
        buffer (final after fb_head), then the rest (final after fb_rest)."""
        h = self.head_end
        return [self.grad[:h], self.grad[h:]] if 0 < h < self.grad.numel() else [self.grad]

    def _allreduce_async(self, i):
        """Start the all-reduce of gradient bucket ``i``.  grad_comm "bf16" (SURVEY.md §5): a bf16 copy of the
        bucket travels (half the bytes per link), summed in bf16 by RCCL and widened back into the f32 master
        gradient by _finish_buckets."""
        import torch.distributed as dist
        bucket = self._grad_buckets()[i]
        if self.grad_comm == "bf16":
            comm = self._comm.get(i)
            if comm is None or comm.numel() != bucket.numel():
                comm = self._comm[i] = torch.empty(bucket.numel(), device=bucket.device, dtype=torch.bfloat16)
            comm.copy_(bucket)
            bucket = comm
        return dist.all_reduce(bucket, group=self.group, async_op=True)

    def _finish_buckets(self, works):
        for w in works:
            w.wait()
        if self.grad_comm == "bf16":
            for i, b in enumerate(self._grad_buckets()):
                b.copy_(self._comm[i])

    def allreduce_grads(self):
        """DDP gradient averaging over the flat f32 gradient (bucket by bucket; sum then / world)."""
        if self._ddp():
            self._finish_buckets([self._allreduce_async(i) for i in range(len(self._grad_buckets()))])
            self.grad.mul_(1.0 / self.world)

    def train_iteration(self, x, y, flow, labels, ant_targets, masks=None):
        """Eager data-parallel iteration with the head bucket's all-reduce overlapped with the backbone
        backward: buffers sync -> fb_head -> all-reduce(head) in flight -> fb_rest -> all-reduce(rest)
        -> wait -> average -> SGD."""
        self.sync_buffers()
        out = self.fb_head(x, y, flow, labels, ant_targets, masks)
        nb = len(self._grad_buckets())
        works = [self._allreduce_async(0)] if self._ddp() and nb > 1 else []
        self.fb_rest()
        if self._ddp():
            works.append(self._allreduce_async(nb - 1))
            self._finish_buckets(works)
            self.grad.mul_(1.0 / self.world)
        self.optimizer_step()
        return out

    def _optimizer_launch(self, first):
        h = self.hp
        ops.sgd(self.flat, self.grad, self.mom, h["lr"], h["momentum"], h["dampening"], h["weight_decay"],
                h["nesterov"], first=first)
        self._refresh_packs()
        self.counter.add_(1)

    def _after_step(self):
        self.steps += 1
        # the kernels wrote the parameters behind autograd's back: bump their version counters so the
        # eval-mode modules re-derive their cached packs (svk.pack.PackCache)
        for p in self.params.values():
            increment_version(p)

    def optimizer_step(self):
        self._optimizer_launch(first=self.steps == 0)
        self._after_step()

    def step(self, x, y, flow, labels, ant_targets, masks=None):
        """One train_model iteration (train_evp.py:473-515): returns (loss [2], logits, anticipation).
        After capture() with these same input tensors, the iteration replays as one HIP graph."""
        if self.graph is not None and masks is None and self._static == (x, y, flow, labels, ant_targets):
            return self._replay()
        return self.train_iteration(x, y, flow, labels, ant_targets, masks)

    # ---- HIP graph capture ----------------------------------------------------------------------
    def capture(self, x, y, flow, labels, ant_targets):
        """Capture one full iteration (forward, backward, SGD, re-pack) over these input tensors as a
        HIP graph (torch.cuda.CUDAGraph drives hipStreamBeginCapture).  The ~700 kernel launches of a
        step then cost one graph launch.  With DDP no collective is captured: three graphs (fb_head,
        fb_rest, averaging + optimizer) replay around the eager BN-buffer broadcast and the two bucket
        all-reduces, the head bucket's overlapping fb_rest.  Needs at least one eager step first
        (momentum buffer initialised)."""
        if self.steps == 0:
            raise SvkError("EVPTrainStep.capture: run one eager step first")
        self._static = (x, y, flow, labels, ant_targets)
        ddp = self._ddp()
        bns = [self.model.head.linear_fuse.bn] + [getattr(self.model.flow_encoder, f"bn{i}") for i in range(1, 5)]
        saved = [(bn.running_mean.clone(), bn.running_var.clone(), bn.num_batches_tracked.clone()) for bn in bns]
        s = torch.cuda.Stream(device=self.dev)
        s.wait_stream(torch.cuda.current_stream(self.dev))
        with torch.cuda.stream(s):        # warm the allocator's private pool outside the capture
            self.forward_backward(*self._static)
        torch.cuda.current_stream(self.dev).wait_stream(s)
        with torch.no_grad():             # the warm-up pass must not count as a BatchNorm update
            for bn, (rm, rv, nb) in zip(bns, saved):
                bn.running_mean.copy_(rm)
                bn.running_var.copy_(rv)
                bn.num_batches_tracked.copy_(nb)
        self.graph_rest = self.graph_opt = None
        self.graph = torch.cuda.CUDAGraph()
        if not ddp:
            with torch.cuda.graph(self.graph):
                self._gout = self.forward_backward(*self._static)
                self._optimizer_launch(first=False)
            return self
        pool = torch.cuda.graph_pool_handle()
        # thread-local capture: the process group's watchdog thread polls the completion events of earlier
        # collectives (hipEventQuery) at any time, which a global-mode capture treats as an illegal call
        # from another thread and aborts on (seen on MI355X as "operation not permitted when stream is
        # capturing" in the watchdog).  The captured work itself never calls into RCCL.
        torch.cuda.synchronize(self.dev)
        mode = dict(pool=pool, capture_error_mode="thread_local")
        with torch.cuda.graph(self.graph, **mode):
            self._gout = self.fb_head(*self._static)
        self.graph_rest = torch.cuda.CUDAGraph()
        with torch.cuda.graph(self.graph_rest, **mode):
            self.fb_rest()
        self.graph_opt = torch.cuda.CUDAGraph()
        with torch.cuda.graph(self.graph_opt, **mode):
            self.grad.mul_(1.0 / self.world)
            self._optimizer_launch(first=False)
        return self

    def _replay(self):
        if self.graph_rest is None:
            self.graph.replay()
        else:
            self.sync_buffers()
            self.graph.replay()
            nb = len(self._grad_buckets())
            works = [self._allreduce_async(0)] if nb > 1 else []
            self.graph_rest.replay()
            works.append(self._allreduce_async(nb - 1))
            self._finish_buckets(works)
            self.graph_opt.replay()
        self._after_step()
        return self._gout


# ---------------------------------------------------------------------------------------------------
class EVPAutograd(EVPTrainStep):
    """The train-mode ``MixVisionTransformerEVP.forward`` of the drop-in surface as ONE autograd node
    over the same forward / backward kernels as EVPTrainStep, so the reference's own loop runs unchanged
    (train_evp.py:473-515, finetune_evp.py:396/509): ``model.train()``, ``autocast(float16)`` forward ->
    (y [B, 7], y_ant [B, 7]), torch criteria, ``scaler.scale(loss).backward()``, ``scaler.step(optimizer)``
    with torch's own SGD over the reference's parameter groups.

    * The trainable parameters are views into one flat f32 buffer (torch's optimizer updates them in
      place); their ``.grad`` stay autograd's (the node returns one gradient per parameter; the freeze
      rule of train_evp.py:379-382 is checked, not imposed).  Parameter updates are seen through the
      version counters: the compute-dtype weight packs are re-derived before the next forward, and a
      change to a frozen backbone parameter rebuilds the trainer.
    * Compute dtype = the autocast region's (svk.default_dtype(): f16 under autocast(float16), as the
      reference trains) or ``model.svk_dtype``; f32 outside autocast.
    * Train-mode semantics as EVPTrainStep: DropPath / Dropout2d masks from the device counter (a new
      draw every forward), BatchNorm batch statistics with the running-stat update in the forward.
    * Each forward keeps its own saved activations in the node (several forwards before a backward —
      gradient accumulation — are independent)."""

    BIND_GRADS = False

    def __init__(self, model, dtype, counter=None):
        # the mask stream follows torch's seed (torch.manual_seed, as the reference's DropPath / Dropout2d
        # draws do), and a rebuilt trainer continues the previous one's device step count instead of
        # replaying the masks of step 0
        super().__init__(model, dtype=dtype, drop=True, seed=torch.initial_seed() & 0x7FFFFFFF)
        if counter is not None:
            self.counter.copy_(counter)
        self.names = list(self.params)
        self._snap()

    def _snap(self):
        self._ver_tr = [self.params[n]._version for n in self.names]
        self._ver_fz = [p._version for n, p in self.model.named_parameters() if not is_trainable(n)]

    def frozen_changed(self):
        return [p._version for n, p in self.model.named_parameters() if not is_trainable(n)] != self._ver_fz

    def ensure_fresh(self):
        if [self.params[n]._version for n in self.names] != self._ver_tr:
            self._refresh_packs()
            self._snap()

    def forward_saved(self, x, y, flow):
        B = x.numel() // (3 * 224 * 224)
        masks = self.make_masks(B)
        self.counter.add_(1)                         # fresh DropPath / Dropout2d draws next forward
        sv, logits, ant = self._forward(x, y, flow, masks)
        self._update_bn_running(sv)                  # nn.BatchNorm2d updates its running stats in forward
        return sv, logits, ant

    def backward_grads(self, sv, dlogits, dant):
        self.grad.zero_()
        self.conv_scratch.zero_()
        self._backward_rest(sv, self._backward_head(sv, dlogits, dant))
        self.untab.run(self.conv_scratch, self.grad)
        return [self.grad[self.off[n]:self.off[n] + self.params[n].numel()].view_as(self.params[n]).clone()
                for n in self.names]


class _EVPFn(torch.autograd.Function):
    @staticmethod
    def forward(ctx, tr, x, y, flow, *params):
        sv, logits, ant = tr.forward_saved(x, y, flow)
        ctx.tr, ctx.sv = tr, sv
        ctx.shape = tuple(logits.shape)
        return logits, ant

    @staticmethod
    @torch.autograd.function.once_differentiable
    def backward(ctx, g_logits, g_ant):
        tr, sv = ctx.tr, ctx.sv
        ctx.sv = None
        z = lambda g: (torch.zeros(ctx.shape, device=tr.dev, dtype=torch.float32) if g is None
                       else g.float().contiguous())
        grads = tr.backward_grads(sv, z(g_logits), z(g_ant))
        return (None, None, None, None) + tuple(grads)


def evp_trainer(model, dtype):
    t = model.__dict__.get("_svk_evp_autograd")
    if t is None or t.dt != dtype or t.frozen_changed():
        t = EVPAutograd(model, dtype, counter=None if t is None else t.counter)
        model.__dict__["_svk_evp_autograd"] = t
    return t


def autograd_forward(model, x, y, flow, dtype):
    """Train-mode MixVisionTransformerEVP.forward(x, y, flow) -> (y [B, 7], y_ant [B, 7]) f32, one autograd
    node (EVPAutograd)."""
    for t in (x, y, flow):
        if t is None:
            raise SvkError("MixVisionTransformerEVP train mode: the svk path trains with the optical-flow input "
                           "(train_evp.py:495 always passes it)")
        if not t.is_cuda:
            raise SvkError(f"MixVisionTransformerEVP: inputs must be on the GPU (got {t.device}); there is no CPU path")
    tr = evp_trainer(model, dtype)
    tr.ensure_fresh()
    return _EVPFn.apply(tr, x, y, flow, *[tr.params[n] for n in tr.names])
