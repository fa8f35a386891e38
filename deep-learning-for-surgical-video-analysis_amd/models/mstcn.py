"""MS-TCN temporal model — MI355X build (drop-in for the reference's models/mstcn.py).

``MultiStageModel_S`` / ``SingleStageModel`` / ``DilatedResidualLayer`` keep the
reference's constructor signatures, submodule names and ``state_dict`` keys
(mstcn.py:94-214).  Arithmetic: the video's feature sequence is consumed
time-major ([T, f_dim], the LFB row layout — the reference's ``[1, f_dim, T]`` input
is a transposed view of exactly that), the 1x1 convs are MFMA GEMMs, each dilated
residual layer (dilated k=3 conv + ReLU + 1x1 conv + residual) is ONE svk kernel, and
the inter-stage softmax over classes is one kernel.  Everything runs in f32 (the
reference path is f32; this model is HBM/launch-bound, not MFMA-bound).

Output: ``[stages, B, classes, T]`` like the reference, returned as a view of the
time-major [stages, B, T, classes] buffer the kernels write.
"""
import copy
import math

import torch
import torch.nn as nn

from svk import ops, temporal
from svk.pack import get_packed
from ._common import check_inference



def _w1x1(conv):
    return conv.weight.detach().float()[:, :, 0].contiguous(), conv.bias.detach().float().contiguous()


class DilatedResidualLayer(nn.Module):
    """(mstcn.py:181-214)."""

    def __init__(self, dilation, in_channels, out_channels, causal_conv=False, kernel_size=3):
        super().__init__()
        self.causal_conv = causal_conv
        self.dilation = dilation
        self.kernel_size = kernel_size
        pad = dilation * (kernel_size - 1) if causal_conv else dilation
        self.conv_dilated = nn.Conv1d(in_channels, out_channels, kernel_size, padding=pad, dilation=dilation)
        self.conv_1x1 = nn.Conv1d(out_channels, out_channels, 1)
        self.dropout = nn.Dropout()

    def _pack(self, dt):
        wdT = self.conv_dilated.weight.detach().float().permute(2, 1, 0).contiguous()   # [3][F_in][F_out]
        w1, b1 = _w1x1(self.conv_1x1)
        return dict(wdT=wdT, bd=self.conv_dilated.bias.detach().float().contiguous(), w1T=w1.t().contiguous(), b1=b1)

    def forward_tm(self, x, tiles=None):
        """x [T, F] time-major f32 -> [T, F] (``tiles``: x is a ragged batch of videos, ops.mstcn_tiles)."""
        p = get_packed(self, torch.float32, self._pack)
        return ops.mstcn_layer(x, p["wdT"], p["bd"], p["w1T"], p["b1"], self.dilation, self.causal_conv, tiles=tiles)

    def forward(self, x):
        """Reference signature: x [B, F, T] -> [B, F, T]."""
        check_inference(self, x)
        return torch.stack([self.forward_tm(xb.t().float().contiguous()).t() for xb in x], 0)


class SingleStageModel(nn.Module):
    """(mstcn.py:153-178)."""

    def __init__(self, num_layers, num_f_maps, dim, num_classes, causal_conv=False):
        super().__init__()
        if num_layers > 0 and num_f_maps > 64:
            raise ValueError("SingleStageModel: the svk dilated-residual kernel supports num_f_maps <= 64")
        self.conv_1x1 = nn.Conv1d(dim, num_f_maps, 1)
        self.layers = nn.ModuleList([copy.deepcopy(DilatedResidualLayer(2 ** i, num_f_maps, num_f_maps,
                                                                        causal_conv=causal_conv))
                                     for i in range(num_layers)])
        self.conv_out_classes = nn.Conv1d(num_f_maps, num_classes, 1)

    def _pack(self, dt):
        wi, bi = _w1x1(self.conv_1x1)
        wo, bo = _w1x1(self.conv_out_classes)
        return dict(wi=wi, bi=bi, wo=wo, bo=bo)

    def forward_tm(self, x, out=None, tiles=None):
        """x [T, dim] time-major f32 -> class logits [T, classes] (written into ``out`` if given)."""
        p = get_packed(self, torch.float32, self._pack)
        h = ops.gemm(x, p["wi"], p["bi"])
        for layer in self.layers:
            h = layer.forward_tm(h, tiles)
        return ops.gemm(h, p["wo"], p["bo"], out=out)

    def forward(self, x):
        check_inference(self, x)
        return torch.stack([self.forward_tm(xb.t().float().contiguous()).t() for xb in x], 0)


class MultiStageModel_S(nn.Module):
    """(mstcn.py:94-130)."""

    def __init__(self, mstcn_stages, mstcn_layers, mstcn_f_maps, mstcn_f_dim, out_features, mstcn_causal_conv):
        self.num_stages = mstcn_stages
        self.num_layers = mstcn_layers
        self.num_f_maps = mstcn_f_maps
        self.dim = mstcn_f_dim
        self.num_classes = out_features
        self.causal_conv = mstcn_causal_conv
        print(f"num_stages_classification: {self.num_stages}, num_layers: {self.num_layers}, num_f_maps:"
              f" {self.num_f_maps}, dim: {self.dim}")
        super().__init__()
        self.stage1_phase = SingleStageModel(self.num_layers, self.num_f_maps, self.dim, self.num_classes,
                                             causal_conv=self.causal_conv)
        self.stages = nn.ModuleList([copy.deepcopy(SingleStageModel(self.num_layers, self.num_f_maps,
                                                                    self.num_classes, self.num_classes,
                                                                    causal_conv=self.causal_conv))
                                     for s in range(self.num_stages - 1)])
        self.smoothing = False

    def forward_tm(self, x, tiles=None):
        """x [T, f_dim] (f32, time-major) -> [stages, T, classes] time-major logits."""
        T = x.shape[0]
        out = torch.empty(self.num_stages, T, self.num_classes, device=x.device, dtype=torch.float32)
        self.stage1_phase.forward_tm(x, out=out[0], tiles=tiles)
        for s, stage in enumerate(self.stages):
            prob = ops.softmax_rows(out[s])                       # softmax over classes (mstcn.py:126)
            stage.forward_tm(prob, out=out[s + 1], tiles=tiles)
        return out

    def forward_videos(self, feats, lengths):
        """Eval forward of a ragged batch of videos in one pass (one launch per layer for all of them).

        ``feats`` [sum(lengths), f_dim]: the videos' feature rows concatenated time-major in order —
        the layout of the long-range feature bank the callers slice per video (trans_SV_output.py:251-291,
        tecno.py:80-91).  Returns [stages, sum(lengths), classes] time-major logits; video v's rows
        ``out[:, o_v:o_v + T_v]`` equal ``self(feats[o_v:o_v + T_v].t()[None])`` (as [S, 1, C, T_v]
        after ``.permute(0, 2, 1)[:, None]``).  See ``split_videos``."""
        check_inference(self, feats)
        if feats.dim() != 2 or feats.shape[0] != sum(int(t) for t in lengths):
            raise ValueError("forward_videos: feats must be [sum(lengths), f_dim]")
        x = feats if (feats.dtype == torch.float32 and feats.is_contiguous()) else feats.float().contiguous()
        return self.forward_tm(x, tiles=ops.mstcn_tiles(lengths, x.device))

    @staticmethod
    def split_videos(out_tm, lengths):
        """forward_videos output -> per-video [stages, 1, classes, T_v] views (the reference's layout)."""
        res, o = [], 0
        for T in lengths:
            res.append(out_tm[:, o:o + int(T)].permute(0, 2, 1).unsqueeze(1))
            o += int(T)
        return res

    def forward(self, x):
        """x [B, f_dim, T] -> [stages, B, classes, T] (mstcn.py:122-130).  Train mode (tecno.py:195):
        dropout active, forward/backward on the svk training kernels (svk.temporal)."""
        if self.training:
            return temporal.autograd_forward(self, x)
        check_inference(self, x)
        per = []
        for xb in x:                                   # batch of videos (the reference uses B = 1)
            xt = xb.t()                                # [T, f_dim]; a view when x = lfb.transpose(2, 1)
            if xt.dtype != torch.float32 or xt.stride(1) != 1:
                xt = xt.float().contiguous()
            per.append(self.forward_tm(xt))
        out = torch.stack(per, dim=1) if len(per) > 1 else per[0].unsqueeze(1)   # [S, B, T, C]
        return out.permute(0, 1, 3, 2)

    @staticmethod
    def add_model_specific_args(parser):  # pragma: no cover
        g = parser.add_argument_group(title="mstcn reg specific args options")
        g.add_argument("--mstcn_stages", default=4, type=int)
        g.add_argument("--mstcn_layers", default=10, type=int)
        g.add_argument("--mstcn_f_maps", default=64, type=int)
        g.add_argument("--mstcn_f_dim", default=2048, type=int)
        g.add_argument("--mstcn_causal_conv", action="store_true")
        return parser


class Mamba(nn.Module):
    """Selective state-space block with the parameter names, shapes and initialisation of
    ``mamba_ssm.Mamba`` (v1, mamba_simple.py) — the module the reference imports at mstcn.py:9 and
    stacks at mstcn.py:316-322 — so checkpoints written by the reference load strictly.  The forward is
    MI355X-native: in_proj / x_proj / out_proj are MFMA GEMMs (f32), the causal depthwise conv + SiLU is
    ``svk_mamba_conv_silu`` and the selective scan (dt projection, softplus, D skip and silu(z) gate
    fused) is ``svk_mamba_scan``.  ``forward_tm`` adds the block's residual in out_proj's epilogue
    (CausalMambaModel: ``x = x + blk(x)``, mstcn.py:335)."""

    def __init__(self, d_model, d_state=16, d_conv=4, expand=2, dt_rank="auto", dt_min=0.001, dt_max=0.1,
                 dt_init="random", dt_scale=1.0, dt_init_floor=1e-4, conv_bias=True, bias=False,
                 use_fast_path=True, layer_idx=None, device=None, dtype=None):
        super().__init__()
        self.d_model, self.d_state, self.d_conv, self.expand = d_model, d_state, d_conv, expand
        self.d_inner = int(expand * d_model)
        self.dt_rank = math.ceil(d_model / 16) if dt_rank == "auto" else dt_rank
        self.layer_idx = layer_idx
        self.in_proj = nn.Linear(d_model, self.d_inner * 2, bias=bias)
        self.conv1d = nn.Conv1d(self.d_inner, self.d_inner, d_conv, groups=self.d_inner, padding=d_conv - 1,
                                bias=conv_bias)
        self.activation = "silu"
        self.act = nn.SiLU()
        self.x_proj = nn.Linear(self.d_inner, self.dt_rank + d_state * 2, bias=False)
        self.dt_proj = nn.Linear(self.dt_rank, self.d_inner, bias=True)
        std = self.dt_rank ** -0.5 * dt_scale
        if dt_init == "constant":
            nn.init.constant_(self.dt_proj.weight, std)
        else:
            nn.init.uniform_(self.dt_proj.weight, -std, std)
        dt = torch.exp(torch.rand(self.d_inner) * (math.log(dt_max) - math.log(dt_min)) + math.log(dt_min))
        dt = dt.clamp(min=dt_init_floor)
        with torch.no_grad():
            self.dt_proj.bias.copy_(dt + torch.log(-torch.expm1(-dt)))
        A = torch.arange(1, d_state + 1, dtype=torch.float32).repeat(self.d_inner, 1)
        self.A_log = nn.Parameter(torch.log(A))
        self.D = nn.Parameter(torch.ones(self.d_inner))
        self.out_proj = nn.Linear(self.d_inner, d_model, bias=bias)

    def _pack(self, dt):
        f = lambda t: t.detach().float().contiguous()
        return dict(w_in=f(self.in_proj.weight), b_in=None if self.in_proj.bias is None else f(self.in_proj.bias),
                    conv_w=f(self.conv1d.weight[:, 0, :]),
                    conv_b=None if self.conv1d.bias is None else f(self.conv1d.bias),
                    w_x=f(self.x_proj.weight), w_dt=f(self.dt_proj.weight), b_dt=f(self.dt_proj.bias),
                    a_neg=(-torch.exp(self.A_log.detach().float())).contiguous(), d_skip=f(self.D),
                    w_out=f(self.out_proj.weight),
                    b_out=None if self.out_proj.bias is None else f(self.out_proj.bias))

    def forward_tm(self, x, B, T, residual=None, ragged=None):
        """x [B*T, d_model] f32 time-major -> out_proj(y) (+ residual) [B*T, d_model].  ``ragged``
        (ops.mamba_ragged): x is a ragged batch of videos concatenated time-major (B, T unused)."""
        p = get_packed(self, torch.float32, self._pack)
        di = self.d_inner
        xz = ops.gemm(x, p["w_in"], p["b_in"])                           # [BT, 2 Di]
        xc = ops.mamba_conv_silu(xz[:, :di], p["conv_w"], p["conv_b"], B, T, ragged=ragged)
        xdbl = ops.gemm(xc, p["w_x"])                                     # [BT, R + 2N]
        y = ops.mamba_scan(xc, xdbl, xz[:, di:], p["w_dt"], p["b_dt"], p["a_neg"], p["d_skip"], B, T, ragged=ragged)
        return ops.gemm(y, p["w_out"], p["b_out"], residual=residual)

    def forward(self, hidden_states):
        """mamba_ssm signature: [B, L, d_model] -> [B, L, d_model]."""
        check_inference(self, hidden_states)
        B, L, Dm = hidden_states.shape
        x = hidden_states.float().contiguous().view(B * L, Dm)
        return self.forward_tm(x, B, L).view(B, L, Dm)


class CausalMambaModel(nn.Module):
    """(mstcn.py:282-343).  Same constructor, submodule names and state_dict keys as the reference
    (``in_proj``, ``blocks.{i}`` = Mamba v1 blocks, ``dropout``, ``norm``, ``head``); the reference raises
    ImportError without ``mamba_ssm`` (mstcn.py:301-302) — this build carries its own selective-scan
    kernels instead.  Eval-mode forward: x [B, f_dim, T] -> [1, B, classes, T], all time-major f32:
    in_proj GEMM, per block (GEMM, conv+SiLU, GEMM, scan, GEMM + residual), LayerNorm, head GEMM.
    Train mode (tecno.py:153, 195): dropout after every block, forward and backward on the svk
    training kernels (svk.temporal: selective-scan / conv+SiLU backward kernels, f32 MFMA GEMMs)."""

    def __init__(self, mstcn_stages, mstcn_layers, mstcn_f_maps, mstcn_f_dim, out_features, mstcn_causal_conv,
                 mamba_d_state=64, mamba_d_conv=4, mamba_expand=2, mamba_dropout=0.1):
        super().__init__()
        self.num_stages = mstcn_stages
        self.num_layers = mstcn_layers
        self.num_f_maps = mstcn_f_maps
        self.dim = mstcn_f_dim
        self.num_classes = out_features
        self.causal_conv = mstcn_causal_conv
        self.mamba_d_state = mamba_d_state
        self.mamba_d_conv = mamba_d_conv if 2 <= mamba_d_conv <= 4 else 4     # mstcn.py:313
        self.mamba_expand = mamba_expand
        if mamba_d_state not in (16, 32, 64):
            raise ValueError("CausalMambaModel: the svk selective scan supports d_state in {16, 32, 64}")
        self.in_proj = nn.Linear(self.dim, self.num_f_maps)
        self.blocks = nn.ModuleList([Mamba(d_model=self.num_f_maps, d_state=self.mamba_d_state,
                                           d_conv=self.mamba_d_conv, expand=self.mamba_expand)
                                     for _ in range(self.num_layers)])
        if self.blocks and self.blocks[0].dt_rank > 16:
            raise ValueError("CausalMambaModel: the svk selective scan supports dt_rank <= 16 (f_maps <= 256)")
        self.dropout = nn.Dropout(mamba_dropout)
        self.norm = nn.LayerNorm(self.num_f_maps)
        self.head = nn.Linear(self.num_f_maps, self.num_classes)

    def _pack(self, dt):
        f = lambda t: t.detach().float().contiguous()
        return dict(w_in=f(self.in_proj.weight), b_in=f(self.in_proj.bias), g=f(self.norm.weight),
                    b=f(self.norm.bias), w_h=f(self.head.weight), b_h=f(self.head.bias))

    def forward(self, x):
        if self.training:                                                 # tecno.py:195 (svk.temporal)
            return temporal.autograd_forward(self, x)
        check_inference(self, x)
        B, C, T = x.shape
        p = get_packed(self, torch.float32, self._pack)
        xt = x.transpose(1, 2)                                            # [B, T, C]
        if xt.dtype != torch.float32 or not xt.is_contiguous():
            xt = xt.float().contiguous()
        h = ops.gemm(xt.view(B * T, C), p["w_in"], p["b_in"])
        for blk in self.blocks:
            h = blk.forward_tm(h, B, T, residual=h)                       # x = x + blk(x); dropout: eval identity
        h = ops.layernorm(h, p["g"], p["b"], self.norm.eps)
        logits = ops.gemm(h, p["w_h"], p["b_h"])                          # [B*T, classes]
        return logits.view(B, T, self.num_classes).permute(0, 2, 1).unsqueeze(0)

    def forward_videos(self, feats, lengths):
        """Eval forward of a ragged batch of videos in one pass (one launch per kernel for all of them).

        ``feats`` [sum(lengths), f_dim]: the videos' feature rows concatenated time-major (the feature
        bank layout the callers slice per video, tecno.py:80-91).  Returns [sum(lengths), classes]
        time-major logits; video v's rows equal ``self(feats[o_v:o_v + T_v].t()[None])`` (see
        ``split_videos``): the causal conv and the scan restart at every video's first frame."""
        check_inference(self, feats)
        if feats.dim() != 2 or feats.shape[0] != sum(int(t) for t in lengths):
            raise ValueError("forward_videos: feats must be [sum(lengths), f_dim]")
        x = feats if (feats.dtype == torch.float32 and feats.is_contiguous()) else feats.float().contiguous()
        p = get_packed(self, torch.float32, self._pack)
        rg = ops.mamba_ragged(lengths, x.device)
        h = ops.gemm(x, p["w_in"], p["b_in"])
        for blk in self.blocks:
            h = blk.forward_tm(h, 1, x.shape[0], residual=h, ragged=rg)
        h = ops.layernorm(h, p["g"], p["b"], self.norm.eps)
        return ops.gemm(h, p["w_h"], p["b_h"])

    @staticmethod
    def split_videos(out_tm, lengths):
        """forward_videos output -> per-video [1, 1, classes, T_v] views (the reference's layout)."""
        res, o = [], 0
        for T in lengths:
            res.append(out_tm[o:o + int(T)].t().unsqueeze(0).unsqueeze(0))
            o += int(T)
        return res
