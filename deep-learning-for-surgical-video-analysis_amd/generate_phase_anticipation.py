"""Drop-in for the reference's top-level ``generate_phase_anticipation.py`` (imported by
trans_SV_output.py:14 for ``plot_phase_anticipation``; its ``generate_anticipation_gt`` builds the
anticipation regression targets, generate_phase_anticipation.py:10-34).

The targets come from the svk HIP kernel ``svk_anticipation_gt`` (one thread per phase series, the
reference's backward recurrence in double precision, bit-exact to the reference function:
tests/test_labels_gpu.py).  The reference computes on CPU LongTensors and returns CPU float tensors; the
drop-in accepts the same CPU input, runs the kernel on the current GPU and hands back a tensor on the
input's device.  There is no CPU path: without a GPU these functions raise.
"""
import torch

from svk import SvkError
from svk.labels import generate_anticipation_gt as _gpu_anticipation_gt


def _on_gpu(t):
    if t.is_cuda:
        return t
    if not torch.cuda.is_available():
        raise SvkError("generate_anticipation_gt: the MI355X build computes the targets on the GPU "
                       "(svk_anticipation_gt) and no GPU is visible; there is no CPU path")
    return t.to("cuda")


def generate_anticipation_gt(phases, horizon):
    """phases [P, T] one-hot phase presence (LongTensor) -> [T, P] float32 targets in [0, 1]
    (generate_phase_anticipation.py:33-34)."""
    phases = torch.as_tensor(phases)
    out = _gpu_anticipation_gt(_on_gpu(phases), horizon)
    return out if phases.is_cuda else out.cpu()


def generate_anticipation_gt_onephase(phase_code, horizon):
    """One phase's presence signal [T] -> [T] float32 targets (generate_phase_anticipation.py:10-30)."""
    phase_code = torch.as_tensor(phase_code)
    return generate_anticipation_gt(phase_code.reshape(1, -1), horizon)[:, 0]


def plot_phase_anticipation(save_path, phase_gt, phase_pred=None):
    """One subplot per phase: ground truth (red) and optional prediction (blue) over frames, y ticks
    0 / 0.5 / >1, saved at 120 dpi (generate_phase_anticipation.py:37-52).  Host-side plotting."""
    import matplotlib.pyplot as plt        # the caller's backend, as the reference (no backend switch)

    def host(a):
        return a.detach().cpu().numpy() if isinstance(a, torch.Tensor) else a

    gt, pred = host(phase_gt), host(phase_pred) if phase_pred is not None else None
    n = gt.shape[-1]
    plt.clf()
    fig = plt.figure(figsize=(30, 2 * n))
    for i in range(n):
        plt.subplot(n, 1, i + 1)
        plt.plot(range(len(gt[:, i])), gt[:, i], color="red", linewidth=1)
        if pred is not None:
            plt.plot(range(len(pred[:, i])), pred[:, i], color="blue", linewidth=1)
        plt.ylabel(str(i))
        plt.yticks([0, 0.5, 1], ["0", "0.5", ">1"])
    plt.xlabel("frame")
    plt.savefig(save_path, dpi=120, bbox_inches="tight")
    plt.close(fig)
