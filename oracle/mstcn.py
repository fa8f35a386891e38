"""Functional CPU restatement of mstcn.MultiStageModel_S (oracle).

State-dict keys are those of the reference module: ``stage1_phase.*`` and
``stages.{s}.*``, each SingleStageModel holding ``conv_1x1``, ``layers.{l}.conv_dilated``,
``layers.{l}.conv_1x1`` and ``conv_out_classes``.
"""
import torch
import torch.nn.functional as F


def dilated_residual_layer(x, sd, p, dilation, causal):
    """DilatedResidualLayer.forward (mstcn.py:208-214); causal = pad 2d both sides, trim last 2d (:193-198, 211)."""
    pad = dilation * 2 if causal else dilation
    out = F.relu(F.conv1d(x, sd[p + ".conv_dilated.weight"], sd[p + ".conv_dilated.bias"],
                          padding=pad, dilation=dilation))
    if causal:
        out = out[:, :, :-(dilation * 2)]
    out = F.conv1d(out, sd[p + ".conv_1x1.weight"], sd[p + ".conv_1x1.bias"])
    return x + out


def single_stage(x, sd, p, num_layers, causal):
    """SingleStageModel.forward (mstcn.py:173-178)."""
    out = F.conv1d(x, sd[p + ".conv_1x1.weight"], sd[p + ".conv_1x1.bias"])
    for l in range(num_layers):
        out = dilated_residual_layer(out, sd, f"{p}.layers.{l}", 2 ** l, causal)
    return F.conv1d(out, sd[p + ".conv_out_classes.weight"], sd[p + ".conv_out_classes.bias"])


def multi_stage_s(x, sd, num_stages, num_layers, causal, dtype=torch.float32):
    """MultiStageModel_S.forward (mstcn.py:122-130): x [1, f_dim, T] -> [S, 1, classes, T]."""
    sd = {k: v.to(dtype) for k, v in sd.items()}
    x = x.to(dtype)
    out = single_stage(x, sd, "stage1_phase", num_layers, causal)
    outputs = [out]
    for s in range(num_stages - 1):
        out = single_stage(F.softmax(out, dim=1), sd, f"stages.{s}", num_layers, causal)
        outputs.append(out)
    return torch.stack(outputs, dim=0)
