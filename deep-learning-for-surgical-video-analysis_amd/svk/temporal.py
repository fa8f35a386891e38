"""Training of the temporal models on the svk kernels — tecno.py:192-259 (and the MS-TCN variant it
keeps commented at tecno.py:155).

The reference trains ``CausalMambaModel`` / ``MultiStageModel_S`` one video per optimizer step: the
video's LFB feature sequence [1, f_dim, T] -> per-stage logits, loss = mean over stages of weighted
CrossEntropy (phase) + SmoothL1 (anticipation), backward, clip_grad_norm_(1.0), AdamW.  Here:

* ``MSTCNTrainer`` / ``MambaTrainer`` own one flat f32 parameter buffer (the nn.Parameters become views
  into it) and one flat gradient buffer, plus the derived layouts the kernels read (packed dilated-conv
  taps, transposed weights for the data-gradient GEMMs, A = -exp(A_log)) refreshed by one gather launch
  (``svk_pack_params``) + ``svk_neg_exp`` after every parameter update;
* ``forward`` / ``backward`` are the explicit forward and backward over the svk kernels (time-major
  [T, C] maps; dilated residual layers, selective scan and causal conv each with a hand-written
  backward kernel; GEMMs and weight gradients on the f32 MFMA path); dropout masks come from the
  counter-based ``svk_keep_mask``;
* ``TemporalTrainStep`` chains forward, ``svk_tecno_loss``, backward, ``svk_grad_sqnorm`` and
  ``svk_adamw`` (clip + AdamW, step count and learning rate on the device) and captures the whole
  step in a HIP graph per sequence length (``step`` replays it);
* the drop-in path: ``model.train(); y = model(x); loss.backward()`` in the reference's own loop runs
  the same forward/backward through one autograd Function per model (``autograd_forward``).
"""
import collections

import torch
from torch.autograd.graph import increment_version

from . import ops
from ._lib import SvkError
from .train import _PackTable


class _WS:
    """Named, shape-checked device buffers (fixed addresses across calls: graph-capture friendly)."""

    def __init__(self, device):
        self.dev = device
        self.bufs = {}

    def get(self, name, shape, dtype=torch.float32, zero=False):
        t = self.bufs.get(name)
        if t is None or t.shape != tuple(shape) or t.dtype != dtype:
            t = torch.empty(shape, device=self.dev, dtype=dtype)
            self.bufs[name] = t
        if zero:
            t.zero_()
        return t


class _Flat:
    """All parameters of ``model`` in one f32 buffer (``p.data`` re-pointed to views) + gradient buffer."""

    def __init__(self, model):
        named = list(model.named_parameters())
        dev = named[0][1].device
        if dev.type != "cuda":
            raise SvkError("svk.temporal: the model must be on a GPU (there is no CPU path)")
        self.dev = dev
        al = lambda k: (k + 3) // 4 * 4          # every parameter starts 16-byte aligned (vector loads)
        total = sum(al(p.numel()) for _, p in named)
        self.flat = torch.zeros(total, device=dev, dtype=torch.float32)
        self.grad = torch.zeros(total, device=dev, dtype=torch.float32)
        self.off, self.params = {}, {}
        o = 0
        with torch.no_grad():
            for n, p in named:
                k = p.numel()
                self.flat[o:o + k].copy_(p.detach().reshape(-1))
                p.data = self.flat[o:o + k].view_as(p)
                self.off[n] = o
                self.params[n] = p
                o += al(k)
        self.total = total
        self._ptrs = {n: p.data_ptr() for n, p in self.params.items()}

    def intact(self):
        return all(p.data_ptr() == self._ptrs[n] for n, p in self.params.items())

    def versions(self):
        return tuple(p._version for p in self.params.values())

    def P(self, name):
        return self.params[name].detach()

    def G(self, name):
        p = self.params[name]
        o = self.off[name]
        return self.grad[o:o + p.numel()].view(p.shape)


class _TrainerBase:
    def __init__(self, model):
        self.model = model
        self.fl = _Flat(model)
        self.dev = self.fl.dev
        self.pt = _PackTable(torch.float32)
        self._build_packs()
        self.pt.finalize(self.dev)
        self._negexp = []            # (A_log name, a_neg buffer)
        self._post_packs()
        self.refresh()

    def _post_packs(self):
        pass

    def _T(self, name):
        """Register a transposed [K, N] copy of the 2-D view of parameter ``name`` ([N, K, (1)])."""
        p = self.fl.params[name]
        N, K = p.shape[0], p.numel() // p.shape[0]
        return self.pt.add(self.fl.off[name], (K, N), (1, K))

    def refresh(self):
        """Re-derive every packed layout from the flat parameters (after each update)."""
        self.pt.run(self.fl.flat)
        for name, buf in self._negexp:
            ops.neg_exp(self.fl.P(name).reshape(-1), out=buf.view(-1))
        self._ver = self.fl.versions()

    def ensure_fresh(self):
        if not self.fl.intact():
            raise SvkError("svk.temporal: a parameter was re-allocated (model.to()/cuda() after the trainer was "
                           "built); build a new trainer")
        if self.fl.versions() != self._ver:
            self.refresh()


# ---------------------------------------------------------------------------------------------------
class MSTCNTrainer(_TrainerBase):
    """MultiStageModel_S (mstcn.py:94-130) with nn.Dropout(0.5) in every DilatedResidualLayer."""

    KEEP = 0.5

    def __init__(self, model):
        self.S = model.num_stages
        self.L = model.num_layers
        self.F = model.num_f_maps
        self.C = model.num_classes
        self.causal = bool(model.causal_conv)
        self.stage_names = ["stage1_phase"] + [f"stages.{s}" for s in range(self.S - 1)]
        super().__init__(model)

    def _build_packs(self):
        self.k_wiT, self.k_woT, self.k_wd, self.k_wdT, self.k_w1T = [], [], [], [], []
        F = self.F
        for sn in self.stage_names:
            self.k_wiT.append(self._T(f"{sn}.conv_1x1.weight"))
            self.k_woT.append(self._T(f"{sn}.conv_out_classes.weight"))
            kd, kdT, k1T = [], [], []
            for l in range(self.L):
                o = self.fl.off[f"{sn}.layers.{l}.conv_dilated.weight"]
                # conv_dilated.weight [F_out][F_in][3]: backward [3][F_out][F_in], forward [3][F_in][F_out]
                kd.append(self.pt.add(o, (3, F, F), (1, 3 * F, 3)))
                kdT.append(self.pt.add(o, (3, F, F), (1, 3, 3 * F)))
                k1T.append(self._T(f"{sn}.layers.{l}.conv_1x1.weight"))
            self.k_wd.append(kd)
            self.k_wdT.append(kdT)
            self.k_w1T.append(k1T)

    def masks(self, T, seed, counter=None):
        n = self.S * self.L * T * self.F
        return ops.keep_mask(n, self.KEEP, seed, self.dev, counter).view(self.S, self.L, T, self.F)

    def forward(self, x, masks, ws, out=None):
        """x [T, f_dim] f32 time-major -> logits [S, T, C] (written into ``out`` if given)."""
        P, pk = self.fl.P, self.pt.tensors
        T = x.shape[0]
        F, C = self.F, self.C
        out = ws.get("out", (self.S, T, C)) if out is None else out
        xin = x
        self._xin = []
        for s, sn in enumerate(self.stage_names):
            self._xin.append(xin)
            Din = xin.shape[1]
            h = ops.gemm(xin, P(f"{sn}.conv_1x1.weight").view(F, Din), P(f"{sn}.conv_1x1.bias"),
                         out=ws.get(f"h{s}_0", (T, F)))
            for l in range(self.L):
                lp = f"{sn}.layers.{l}"
                h, _ = ops.mstcn_layer_train(h, pk[self.k_wdT[s][l]], P(f"{lp}.conv_dilated.bias"),
                                             pk[self.k_w1T[s][l]], P(f"{lp}.conv_1x1.bias"), 2 ** l,
                                             self.causal, masks[s, l], out=ws.get(f"h{s}_{l + 1}", (T, F)),
                                             hidden=ws.get(f"H{s}_{l}", (T, F)))
            ops.gemm(h, P(f"{sn}.conv_out_classes.weight").view(C, F), P(f"{sn}.conv_out_classes.bias"), out=out[s])
            if s + 1 < self.S:
                xin = ops.softmax_rows(out[s], out=ws.get(f"p{s}", (T, C)))
        return out

    def backward(self, dout, masks, ws, need_dx=False):
        """dout [S, T, C] -> parameter gradients += into the flat gradient buffer; returns d x (or None)."""
        P, G, pk = self.fl.P, self.fl.G, self.pt.tensors
        S, F, C = self.S, self.F, self.C
        T = dout.shape[1]
        dnext = None
        dx = None
        for s in range(S - 1, -1, -1):
            sn = self.stage_names[s]
            g = dout[s]
            if dnext is not None:
                g = ops.softmax_rows_bwd(ws.bufs[f"p{s}"], dnext, residual=g, out=ws.get("gs", (T, C)))
            hL = ws.bufs[f"h{s}_{self.L}"]
            ops.gemm_wgrad(g, hL, G(f"{sn}.conv_out_classes.weight").view(C, F), G(f"{sn}.conv_out_classes.bias"))
            dh = ops.gemm(g, pk[self.k_woT[s]], out=ws.get("dh_a", (T, F)))
            other = "dh_b"
            for l in range(self.L - 1, -1, -1):
                lp = f"{sn}.layers.{l}"
                dh = ops.mstcn_layer_bwd(ws.bufs[f"h{s}_{l}"], ws.bufs[f"H{s}_{l}"], masks[s, l], dh,
                                         pk[self.k_wd[s][l]], P(f"{lp}.conv_1x1.weight").view(F, F),
                                         G(f"{lp}.conv_dilated.weight"), G(f"{lp}.conv_dilated.bias"),
                                         G(f"{lp}.conv_1x1.weight").view(F, F), G(f"{lp}.conv_1x1.bias"), 2 ** l,
                                         self.causal, dx=ws.get(other, (T, F)), scratch=ws.get("dpre", (T, F)),
                                         ws=ws.get("bwd_ws", (max(ops.mstcn_bwd_floats(T, F), 1),)))
                other = "dh_a" if other == "dh_b" else "dh_b"
            xin = self._xin[s]
            Din = xin.shape[1]
            ops.gemm_wgrad(dh, xin, G(f"{sn}.conv_1x1.weight").view(F, Din), G(f"{sn}.conv_1x1.bias"))
            if s > 0 or need_dx:
                dnext = ops.gemm(dh, pk[self.k_wiT[s]], out=ws.get(f"dx{s}", (T, Din)))
                if s == 0:
                    dx = dnext
        return dx


# ---------------------------------------------------------------------------------------------------
class MambaTrainer(_TrainerBase):
    """CausalMambaModel (mstcn.py:282-343): in_proj, Mamba blocks with ``x = dropout(x + blk(x))``
    (nn.Dropout(mamba_dropout)), LayerNorm, head."""

    def __init__(self, model):
        self.L = model.num_layers
        self.Fm = model.num_f_maps
        self.C = model.num_classes
        self.keep = 1.0 - float(model.dropout.p)
        blk = model.blocks[0] if self.L else None
        self.Di = blk.d_inner if blk else 0
        self.N = blk.d_state if blk else 0
        self.R = blk.dt_rank if blk else 0
        self.K = blk.d_conv if blk else 0
        self.eps = float(model.norm.eps)
        for b in model.blocks:
            if b.in_proj.bias is not None or b.out_proj.bias is not None:
                raise SvkError("svk.temporal: Mamba in_proj / out_proj with bias are not supported (mamba_ssm default: none)")
        super().__init__(model)

    def _build_packs(self):
        self.k_inT = self._T("in_proj.weight")
        self.k_headT = self._T("head.weight")
        self.k_binT, self.k_xT, self.k_dtT, self.k_outT = [], [], [], []
        for l in range(self.L):
            p = f"blocks.{l}."
            self.k_binT.append(self._T(p + "in_proj.weight"))
            self.k_xT.append(self._T(p + "x_proj.weight"))
            self.k_dtT.append(self._T(p + "dt_proj.weight"))
            self.k_outT.append(self._T(p + "out_proj.weight"))

    def _post_packs(self):
        self.a_neg = []
        for l in range(self.L):
            buf = torch.empty(self.Di, self.N, device=self.dev, dtype=torch.float32)
            self.a_neg.append(buf)
            self._negexp.append((f"blocks.{l}.A_log", buf))

    def masks(self, BT, seed, counter=None):
        return ops.keep_mask(self.L * BT * self.Fm, self.keep, seed, self.dev, counter).view(self.L, BT, self.Fm)

    def forward(self, x, B, T, masks, ws, out=None):
        """x [B*T, f_dim] f32 time-major (row b*T + t) -> logits [B*T, C]."""
        P = self.fl.P
        BT = B * T
        Fm, Di, N, R, K = self.Fm, self.Di, self.N, self.R, self.K
        ws.bufs["x_in"] = x                       # per-call: two forwards before their backwards stay apart
        h = ops.gemm(x, P("in_proj.weight"), P("in_proj.bias"), out=ws.get("h0", (BT, Fm)))
        for l in range(self.L):
            p = f"blocks.{l}."
            xz = ops.gemm(h, P(p + "in_proj.weight"), out=ws.get(f"xz{l}", (BT, 2 * Di)))
            xc = ops.mamba_conv_silu(xz[:, :Di], P(p + "conv1d.weight").view(Di, K), P(p + "conv1d.bias"), B, T)
            ws.bufs[f"xc{l}"] = xc
            xdbl = ops.gemm(xc, P(p + "x_proj.weight"), out=ws.get(f"xdbl{l}", (BT, R + 2 * N)))
            y, yss = ops.mamba_scan_train(xc, xdbl, xz[:, Di:], P(p + "dt_proj.weight"), P(p + "dt_proj.bias"),
                                          self.a_neg[l], P(p + "D"), B, T)
            ws.bufs[f"y{l}"], ws.bufs[f"yss{l}"] = y, yss
            o = ops.gemm(y, P(p + "out_proj.weight"), residual=h, out=ws.get("o", (BT, Fm)))
            h = ops.mul_f32(o, masks[l], out=ws.get(f"h{l + 1}", (BT, Fm)))
        hn = ops.layernorm(h, P("norm.weight"), P("norm.bias"), self.eps, out=ws.get("hn", (BT, Fm)))
        return ops.gemm(hn, P("head.weight"), P("head.bias"), out=ws.get("logits", (BT, self.C)) if out is None else out)

    def backward(self, dlogits, B, T, masks, ws, need_dx=False):
        P, G, pk = self.fl.P, self.fl.G, self.pt.tensors
        BT = B * T
        Fm, Di, N, R, K, C = self.Fm, self.Di, self.N, self.R, self.K, self.C
        hn = ws.bufs["hn"]
        ops.gemm_wgrad(dlogits, hn, G("head.weight"), G("head.bias"))
        dhn = ops.gemm(dlogits, pk[self.k_headT], out=ws.get("dhn", (BT, Fm)))
        dh = ops.layernorm_bwd(ws.bufs[f"h{self.L}"], dhn, P("norm.weight"), self.eps, out=ws.get("dh_a", (BT, Fm)),
                               dgamma=G("norm.weight"), dbeta=G("norm.bias"))
        other = "dh_b"
        for l in range(self.L - 1, -1, -1):
            p = f"blocks.{l}."
            h_prev = ws.bufs[f"h{l}"]
            xz, xc, xdbl = ws.bufs[f"xz{l}"], ws.bufs[f"xc{l}"], ws.bufs[f"xdbl{l}"]
            do = ops.mul_f32(dh, masks[l], out=ws.get("do", (BT, Fm)))
            ops.gemm_wgrad(do, ws.bufs[f"y{l}"], G(p + "out_proj.weight"))
            dy = ops.gemm(do, pk[self.k_outT[l]], out=ws.get("dy", (BT, Di)))
            dxz = ws.get("dxz", (BT, 2 * Di))
            dxdbl = ws.get("dxdbl", (BT, R + 2 * N), zero=True)
            dA = ws.get("dA", (Di, N), zero=True)
            du, ds = ops.mamba_scan_bwd(xc, xdbl, xz[:, Di:], P(p + "dt_proj.weight"), P(p + "dt_proj.bias"),
                                        self.a_neg[l], P(p + "D"), ws.bufs[f"yss{l}"], dy, dxz[:, Di:], dxdbl, dA,
                                        G(p + "D"), B, T)
            ops.mul_f32(dA, self.a_neg[l], out=G(p + "A_log"))                 # dA_log = dA * A
            ops.gemm_wgrad(ds, xdbl[:, :R], G(p + "dt_proj.weight"), G(p + "dt_proj.bias"))
            ops.gemm(ds, pk[self.k_dtT[l]], out=dxdbl[:, :R])
            dxc = ops.gemm(dxdbl, pk[self.k_xT[l]], residual=du, out=ws.get("dxc", (BT, Di)))
            ops.gemm_wgrad(dxdbl, xc, G(p + "x_proj.weight"))
            ops.mamba_conv_silu_bwd(xz[:, :Di], P(p + "conv1d.weight").view(Di, K), P(p + "conv1d.bias"), dxc,
                                    dxz[:, :Di], G(p + "conv1d.weight").view(Di, K), G(p + "conv1d.bias"), B, T)
            ops.gemm_wgrad(dxz, h_prev, G(p + "in_proj.weight"))
            dh = ops.gemm(dxz, pk[self.k_binT[l]], residual=do, out=ws.get(other, (BT, Fm)))
            other = "dh_a" if other == "dh_b" else "dh_b"
        x_in = ws.bufs["x_in"]
        ops.gemm_wgrad(dh, x_in, G("in_proj.weight"), G("in_proj.bias"))
        if need_dx:
            return ops.gemm(dh, pk[self.k_inT], out=ws.get("dx", (BT, x_in.shape[1])))
        return None


# ---------------------------------------------------------------------------------------------------
def trainer_for(model):
    t = model.__dict__.get("_svk_trainer")
    if t is None or t.model is not model:
        from models.mstcn import MultiStageModel_S, CausalMambaModel
        if isinstance(model, MultiStageModel_S):
            t = MSTCNTrainer(model)
        elif isinstance(model, CausalMambaModel):
            t = MambaTrainer(model)
        else:
            raise SvkError(f"svk.temporal: no trainer for {type(model).__name__}")
        model.__dict__["_svk_trainer"] = t
    return t


def _seed():
    return int(torch.randint(0, 2 ** 31 - 1, (1,)).item())


class _TemporalFn(torch.autograd.Function):
    """One autograd node for the whole temporal model: forward / backward on the svk kernels."""

    @staticmethod
    def forward(ctx, tr, x, *params):
        tr.ensure_fresh()
        ws = _WS(tr.dev)
        B, Cin, T = x.shape
        xt = x.transpose(1, 2).float().contiguous()                      # [B, T, f_dim] time-major
        ctx.tr, ctx.ws, ctx.B, ctx.T, ctx.Cin = tr, ws, B, T, Cin
        if isinstance(tr, MSTCNTrainer):
            outs, masks = [], []
            for b in range(B):                                             # the reference uses B = 1
                wsb = ws if b == 0 else _WS(tr.dev)
                m = tr.masks(T, _seed())
                o = tr.forward(xt[b], m, wsb, out=torch.empty(tr.S, T, tr.C, device=tr.dev))
                outs.append(o)
                masks.append((wsb, m, tr._xin))
            ctx.per = masks
            tr.last_masks = [m for _, m, _ in masks]
            out = torch.stack(outs, 1)                                     # [S, B, T, C]
            return out.permute(0, 1, 3, 2)
        m = tr.masks(B * T, _seed())
        ctx.masks = m
        tr.last_masks = m
        logits = tr.forward(xt.view(B * T, Cin), B, T, m, ws, out=torch.empty(B * T, tr.C, device=tr.dev))
        return logits.view(B, T, tr.C).permute(0, 2, 1).unsqueeze(0)

    @staticmethod
    @torch.autograd.function.once_differentiable
    def backward(ctx, gout):
        tr = ctx.tr
        tr.fl.grad.zero_()
        need_dx = ctx.needs_input_grad[1]
        dx = None
        if isinstance(tr, MSTCNTrainer):
            g = gout.permute(0, 1, 3, 2).float()                           # [S, B, T, C]
            dxs = []
            for b, (wsb, m, xin) in enumerate(ctx.per):
                tr._xin = xin
                d = tr.backward(g[:, b].contiguous(), m, wsb, need_dx=need_dx)
                dxs.append(d)
            if need_dx:
                dx = torch.stack(dxs, 0).transpose(1, 2)
        else:
            B, T = ctx.B, ctx.T
            g = gout[0].permute(0, 2, 1).float().contiguous().view(B * T, tr.C)
            d = tr.backward(g, B, T, ctx.masks, ctx.ws, need_dx=need_dx)
            if need_dx:
                dx = d.view(B, T, ctx.Cin).transpose(1, 2)
        grads = [tr.fl.G(n).clone() for n in tr.fl.params]
        return (None, dx) + tuple(grads)


def autograd_forward(model, x):
    """Train-mode forward of MultiStageModel_S / CausalMambaModel through one autograd node."""
    if not x.is_cuda:
        raise SvkError(f"{type(model).__name__}: inputs must be on the GPU (got {x.device}); there is no CPU path")
    tr = trainer_for(model)
    return _TemporalFn.apply(tr, x, *tr.fl.params.values())


# ---------------------------------------------------------------------------------------------------
class TemporalTrainStep:
    """One tecno.py optimizer step per call on one video (the reference's batch_size = 1):
    forward, loss (tecno.py:237-254), backward, clip_grad_norm_(grad_clip), AdamW — all svk kernels,
    captured into a HIP graph per sequence length T on first sight (``graphs=True``) and replayed.

    Hyper-parameters default to tecno.py:100, 110-111, 162-168.  ``lr`` lives on the device
    (``set_lr`` for ReduceLROnPlateau)."""

    def __init__(self, model, class_weights=None, lr=1e-4, weight_decay=1e-3, betas=(0.9, 0.999), eps=1e-8,
                 grad_clip=1.0, seed=42, graphs=True, max_graphs=64):
        model.train()
        self.tr = trainer_for(model)
        self.model = model
        self.dev = self.tr.dev
        n = self.tr.fl.total
        self.m = torch.zeros(n, device=self.dev)
        self.v = torch.zeros(n, device=self.dev)
        self.lr = torch.full((1,), float(lr), device=self.dev)
        self.step_t = torch.zeros(1, device=self.dev, dtype=torch.int64)
        self.parts = torch.zeros(ops.NORM_PARTS, device=self.dev)
        self.loss = torch.zeros(3, device=self.dev)
        self.hp = dict(weight_decay=weight_decay, beta1=betas[0], beta2=betas[1], eps=eps, max_norm=grad_clip)
        self.cw = None if class_weights is None else torch.as_tensor(class_weights, dtype=torch.float32).to(self.dev)
        self.seed = int(seed)
        self.graphs = graphs
        # T -> (graph, ws, static inputs): one captured graph per video length, each holding its own
        # activation workspace (MS-TCN S(2L+1)TF f32 + masks, Mamba ~36 KB per frame at 10 blocks, i.e.
        # ~0.2 GB for a 6000-frame video); least-recently-used lengths beyond max_graphs are dropped
        self._g = collections.OrderedDict()
        self._eager = collections.OrderedDict()
        self.max_graphs = int(max_graphs)

    def set_lr(self, lr):
        self.lr.fill_(float(lr))

    def _body(self, x, labels, ant, ws):
        tr = self.tr
        isms = isinstance(tr, MSTCNTrainer)
        T = x.shape[0]
        if isms:
            masks = tr.masks(T, self.seed, self.step_t)
            out = tr.forward(x, masks, ws)                                          # [S, T, C]
        else:
            masks = tr.masks(T, self.seed, self.step_t)
            out = tr.forward(x, 1, T, masks, ws).view(1, T, tr.C)
        _, dlog = ops.tecno_loss(out, labels, ant, self.cw, out=self.loss, dlogits=ws.get("dlogits", tuple(out.shape)))
        tr.fl.grad.zero_()
        if isms:
            tr.backward(dlog, masks, ws)
        else:
            tr.backward(dlog.view(T, tr.C), 1, T, masks, ws)
        ops.grad_sqnorm(tr.fl.grad, self.parts, self.step_t)
        ops.adamw(tr.fl.flat, tr.fl.grad, self.m, self.v, self.lr, self.step_t, self.parts, **self.hp)
        tr.refresh()

    def __call__(self, x, labels, ant):
        """x [T, f_dim] f32 (time-major LFB rows of one video), labels [T] int64, ant [T, P] f32 ->
        device loss [3] = (clc, ant, last-stage correct count), valid until the next call."""
        self.tr.ensure_fresh()
        T = x.shape[0]
        if not self.graphs:
            # eager workspaces are bounded by the same LRU as the captured graphs, in a map of
            # their own so evictions of one kind never drop the other
            ws = self._eager.get(T)
            if ws is None:
                ws = self._eager[T] = _WS(self.dev)
                while len(self._eager) > self.max_graphs:
                    self._eager.popitem(last=False)
            self._eager.move_to_end(T)
            self._body(x, labels, ant, ws)
            self._bump()
            return self.loss
        ent = self._g.get(T)
        if ent is None:
            ws = _WS(self.dev)
            sx = torch.empty_like(x)
            sl = torch.empty_like(labels)
            sa = torch.empty_like(ant)
            sx.copy_(x); sl.copy_(labels); sa.copy_(ant)
            # warm-up on a side stream: allocates every workspace buffer, runs one real step
            s = torch.cuda.Stream()
            s.wait_stream(torch.cuda.current_stream())
            with torch.cuda.stream(s):
                self._body(sx, sl, sa, ws)
            torch.cuda.current_stream().wait_stream(s)
            g = torch.cuda.CUDAGraph()
            with torch.cuda.graph(g):
                self._body(sx, sl, sa, ws)
            self._g[T] = (g, ws, sx, sl, sa)
            while len(self._g) > self.max_graphs:
                self._g.popitem(last=False)
            self._bump()
            return self.loss
        self._g.move_to_end(T)
        g, ws, sx, sl, sa = ent
        sx.copy_(x); sl.copy_(labels); sa.copy_(ant)
        g.replay()
        self._bump()
        return self.loss

    def _bump(self):
        # the kernels updated the parameters in place: bump their version counters so every cached
        # inference pack (svk.pack.get_packed) re-derives, then record the trainer's own view
        for p in self.tr.fl.params.values():
            increment_version(p)
        self.tr._ver = self.tr.fl.versions()


# ---------------------------------------------------------------------------------------------------
class TransformerTrainer(_TrainerBase):
    """adapter_transformer.Transformer.original_forward in train mode (tecno_trans.py:226-292):
    feas = tanh(fc(lfb)) and the build's Transformer2_3_1 (post-LN encoder over the 30-frame window,
    decoder self- then cross-attention, ReLU FFNs; no dropout layers), forward and backward on svk
    kernels (f32 GEMMs / weight gradients, the f32 attention forward and backward, LayerNorm backward)."""

    def __init__(self, model):
        t = model.transformer
        self.len_q = model.len_q
        self.C = model.num_classes
        self.heads = t.encoder.layers[0].self_attn.n_heads if len(t.encoder.layers) else 4
        mha = t.decoder.self_attn
        self.dk, self.dv, self.H = mha.d_k, mha.d_v, mha.n_heads
        self.n_layers = len(t.encoder.layers)
        self.eps = float(mha.layer_norm.eps)
        super().__init__(model)

    def _lin_names(self):
        names = ["fc.weight"]
        mhas = [f"transformer.encoder.layers.{l}.self_attn" for l in range(self.n_layers)]
        mhas += ["transformer.decoder.self_attn", "transformer.decoder.cross_attn"]
        ffns = [f"transformer.encoder.layers.{l}.ffn" for l in range(self.n_layers)] + ["transformer.decoder.ffn"]
        for m in mhas:
            names += [f"{m}.{w}.weight" for w in ("W_Q", "W_K", "W_V", "fc")]
        for f in ffns:
            names += [f"{f}.fc1.weight", f"{f}.fc2.weight"]
        return names

    def _build_packs(self):
        self.kT = {n: self._T(n) for n in self._lin_names()}

    def WT(self, name):
        return self.pt.tensors[self.kT[name + ".weight"]]

    # ---- building blocks: forward saves what the backward needs into ``sv`` ----
    def _lin(self, x, name, act=None, residual=None, out=None):
        P = self.fl.P
        b = self.fl.params.get(name + ".bias")
        return ops.gemm(x, P(name + ".weight"), None if b is None else b.detach(), act=act, residual=residual, out=out)

    def _mha_fwd(self, q_in, kv_in, p, sv):
        P = self.fl.P
        q = self._lin(q_in, p + ".W_Q")
        k = self._lin(kv_in, p + ".W_K")
        v = self._lin(kv_in, p + ".W_V")
        o = ops.attention(q, k, v, self.H, 1.0 / (self.dk ** 0.5))
        pre = self._lin(o, p + ".fc", residual=q_in)
        y = ops.layernorm(pre, P(p + ".layer_norm.weight"), P(p + ".layer_norm.bias"), self.eps)
        sv[p] = (q_in, kv_in, q, k, v, o, pre)
        return y

    def _ffn_fwd(self, x, p, sv):
        P = self.fl.P
        h = self._lin(x, p + ".fc1", act="relu")
        pre = self._lin(h, p + ".fc2", residual=x)
        y = ops.layernorm(pre, P(p + ".layer_norm.weight"), P(p + ".layer_norm.bias"), self.eps)
        sv[p] = (x, h, pre)
        return y

    def forward(self, xt, lf, sv):
        """xt [T, C] (MS-TCN last stage, time-major), lf [T, f_dim] -> [T, 1, C]."""
        P = self.fl.P
        T = xt.shape[0]
        tr = self.model.transformer
        pos = tr.pos_table if self.len_q == tr.len_q else None
        x = ops.window_unfold(xt, self.len_q, pos=pos)
        if pos is None:
            x = ops.add_bcast(x, tr.pos_table)
        pre_f = ops.gemm(lf, P("fc.weight"))                                    # [T, C]
        feas = ops.gemm(lf, P("fc.weight"), act="tanh").view(T, 1, self.C)
        sv["fc"] = (lf, pre_f)
        for l in range(self.n_layers):
            x = self._mha_fwd(x, x, f"transformer.encoder.layers.{l}.self_attn", sv)
            x = self._ffn_fwd(x, f"transformer.encoder.layers.{l}.ffn", sv)
        d = self._mha_fwd(feas, feas, "transformer.decoder.self_attn", sv)
        d = self._mha_fwd(d, x, "transformer.decoder.cross_attn", sv)
        return self._ffn_fwd(d, "transformer.decoder.ffn", sv)

    def _lin_bwd(self, dy, x, name, residual=None, need_dx=True):
        G = self.fl.G
        b = self.fl.params.get(name + ".bias")
        ops.gemm_wgrad(dy, x, G(name + ".weight"), None if b is None else G(name + ".bias"))
        if need_dx:
            return ops.gemm(dy, self.WT(name), residual=residual)
        return None

    def _ln_bwd(self, pre, dy, p):
        return ops.layernorm_bwd(pre, dy, self.fl.P(p + ".layer_norm.weight"), self.eps,
                                 dgamma=self.fl.G(p + ".layer_norm.weight"), dbeta=self.fl.G(p + ".layer_norm.bias"))

    def _mha_bwd(self, dy, p, sv, self_attn):
        q_in, kv_in, q, k, v, o, pre = sv[p]
        dpre = self._ln_bwd(pre, dy, p)
        do = self._lin_bwd(dpre, o, p + ".fc")
        dq, dk, dv = ops.attention_bwd(q, k, v, o, do, self.H, 1.0 / (self.dk ** 0.5))
        dq_in = self._lin_bwd(dq, q_in, p + ".W_Q", residual=dpre)
        if self_attn:
            d = self._lin_bwd(dk, kv_in, p + ".W_K", residual=dq_in)
            return self._lin_bwd(dv, kv_in, p + ".W_V", residual=d), None
        dkv = self._lin_bwd(dk, kv_in, p + ".W_K")
        dkv = self._lin_bwd(dv, kv_in, p + ".W_V", residual=dkv)
        return dq_in, dkv

    def _ffn_bwd(self, dy, p, sv):
        x, h, pre = sv[p]
        G = self.fl.G
        dpre = self._ln_bwd(pre, dy, p)
        ops.gemm_wgrad(dpre, h, G(p + ".fc2.weight"), G(p + ".fc2.bias"))
        dh = ops.gemm(dpre, self.WT(p + ".fc2"), dact="relu", dact_src=h)   # relu'(pre) = [h > 0]
        return self._lin_bwd(dh, x, p + ".fc1", residual=dpre)

    def backward(self, dout, sv):
        """dout [T, 1, C] -> parameter gradients into the flat buffer (the window input is detached at
        tecno_trans.py:271 and the LFB is data: no input gradients)."""
        dd = self._ffn_bwd(dout.contiguous(), "transformer.decoder.ffn", sv)
        dd, denc = self._mha_bwd(dd, "transformer.decoder.cross_attn", sv, self_attn=False)
        dfeas, _ = self._mha_bwd(dd, "transformer.decoder.self_attn", sv, self_attn=True)
        dx = denc
        for l in range(self.n_layers - 1, -1, -1):
            dx = self._ffn_bwd(dx, f"transformer.encoder.layers.{l}.ffn", sv)
            if l > 0:
                dx, _ = self._mha_bwd(dx, f"transformer.encoder.layers.{l}.self_attn", sv, self_attn=True)
            else:                                   # the first layer's input is the (detached) window
                p = f"transformer.encoder.layers.{l}.self_attn"
                q_in, kv_in, q, k, v, o, pre = sv[p]
                dpre = self._ln_bwd(pre, dx, p)
                do = self._lin_bwd(dpre, o, p + ".fc")
                dq, dk, dv = ops.attention_bwd(q, k, v, o, do, self.H, 1.0 / (self.dk ** 0.5))
                for dz, nm in ((dq, ".W_Q"), (dk, ".W_K"), (dv, ".W_V")):
                    self._lin_bwd(dz, q_in, p + nm, need_dx=False)
        lf, pre_f = sv["fc"]
        dpre_f = ops.act_bwd(pre_f, dfeas.reshape(pre_f.shape).contiguous(), "tanh")
        ops.gemm_wgrad(dpre_f, lf, self.fl.G("fc.weight"))


class _TransformerFn(torch.autograd.Function):
    @staticmethod
    def forward(ctx, tr, x, lf, *params):
        tr.ensure_fresh()
        xt = x[0].t().float().contiguous()
        l2 = lf[0].float().contiguous()
        sv = {}
        out = tr.forward(xt, l2, sv)
        ctx.tr, ctx.sv = tr, sv
        return out

    @staticmethod
    @torch.autograd.function.once_differentiable
    def backward(ctx, gout):
        tr = ctx.tr
        tr.fl.grad.zero_()
        tr.backward(gout.float().contiguous(), ctx.sv)
        grads = [tr.fl.G(n).clone() for n in tr.fl.params]
        return (None, None, None) + tuple(grads)


def transformer_autograd_forward(model, x, long_feature):
    """Train-mode Transformer.original_forward(x [1, C, T], long_feature [1, T, f_dim]) -> [T, 1, C]."""
    if not (x.is_cuda and long_feature.is_cuda):
        raise SvkError("Transformer: inputs must be on the GPU; there is no CPU path")
    if x.requires_grad or long_feature.requires_grad:
        raise SvkError("Transformer train mode: input gradients are not built (tecno_trans.py detaches the "
                       "MS-TCN output and the LFB is data)")
    t = model.__dict__.get("_svk_trainer")
    if t is None or t.model is not model:
        t = TransformerTrainer(model)
        model.__dict__["_svk_trainer"] = t
    return _TransformerFn.apply(t, x, long_feature, *t.fl.params.values())
