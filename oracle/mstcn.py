"""Functional CPU restatement of mstcn.MultiStageModel_S (oracle).

State-dict keys are those of the reference module: ``stage1_phase.*`` and
``stages.{s}.*``, each SingleStageModel holding ``conv_1x1``, ``layers.{l}.conv_dilated``,
``layers.{l}.conv_1x1`` and ``conv_out_classes``.
"""
import torch
import torch.nn.functional as F


def dilated_residual_layer(x, sd, p, dilation, causal, mask=None):
    """DilatedResidualLayer.forward (mstcn.py:208-214); causal = pad 2d both sides, trim last 2d (:193-198, 211).
    ``mask`` [1, F, T] (0 or 1/keep): the train-mode nn.Dropout of mstcn.py:213 with a given draw."""
    pad = dilation * 2 if causal else dilation
    out = F.relu(F.conv1d(x, sd[p + ".conv_dilated.weight"], sd[p + ".conv_dilated.bias"],
                          padding=pad, dilation=dilation))
    if causal:
        out = out[:, :, :-(dilation * 2)]
    out = F.conv1d(out, sd[p + ".conv_1x1.weight"], sd[p + ".conv_1x1.bias"])
    if mask is not None:
        out = out * mask
    return x + out


def single_stage(x, sd, p, num_layers, causal, masks=None):
    """SingleStageModel.forward (mstcn.py:173-178)."""
    out = F.conv1d(x, sd[p + ".conv_1x1.weight"], sd[p + ".conv_1x1.bias"])
    for l in range(num_layers):
        out = dilated_residual_layer(out, sd, f"{p}.layers.{l}", 2 ** l, causal,
                                     None if masks is None else masks[l])
    return F.conv1d(out, sd[p + ".conv_out_classes.weight"], sd[p + ".conv_out_classes.bias"])


def multi_stage_s(x, sd, num_stages, num_layers, causal, dtype=torch.float32, masks=None):
    """MultiStageModel_S.forward (mstcn.py:122-130): x [1, f_dim, T] -> [S, 1, classes, T].
    ``masks`` [S, L, T, F] (time-major, as svk draws them): train-mode dropout draws; the state dict
    tensors may require grad (train-mode gradients by autograd in ``dtype``)."""
    sd = {k: v.to(dtype) for k, v in sd.items()}
    x = x.to(dtype)
    mk = None if masks is None else masks.to(dtype).permute(0, 1, 3, 2).unsqueeze(2)   # [S, L, 1, F, T]
    out = single_stage(x, sd, "stage1_phase", num_layers, causal, None if mk is None else mk[0])
    outputs = [out]
    for s in range(num_stages - 1):
        out = single_stage(F.softmax(out, dim=1), sd, f"stages.{s}", num_layers, causal,
                           None if mk is None else mk[s + 1])
        outputs.append(out)
    return torch.stack(outputs, dim=0)


def tecno_loss(y_all, labels, ant_targets, class_w=None):
    """tecno.py:231-254: y_all [S, 1, 2P, T]; CrossEntropyLoss(weight) + SmoothL1Loss averaged over stages.
    Returns (clc_loss, ant_loss)."""
    P = y_all.shape[2] // 2
    S = y_all.shape[0]
    w = None if class_w is None else class_w.to(y_all.dtype)
    clc = 0
    for j in range(S):
        clc = clc + F.cross_entropy(y_all[j, 0, :P].transpose(1, 0), labels, weight=w)
    ant = 0
    for j in range(S):
        ant = ant + F.smooth_l1_loss(y_all[j, 0, P:].transpose(1, 0), ant_targets.to(y_all.dtype))
    return clc / S, ant / S
