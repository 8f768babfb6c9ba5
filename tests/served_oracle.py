"""Shared by the served-pod GPU tests: random full-model weights generated on the
GPU and kept on the host (fp32 for the oracle), and the check of a pod's
``OMNIA_LOGIT_TAP_DIR`` dumps against ``ops.reference.dense_forward``."""
import glob
import math
import os

import torch


def full_llama_weights(mc, seed: int = 7) -> dict:
    """A seeded random full (tp = 1) Llama weight dict, drawn tensor by tensor in
    bf16 on the GPU and moved to the host (bf16)."""
    g = torch.Generator(device="cuda").manual_seed(seed)
    d, D = mc.hidden_size, mc.head_dim

    def init(shape, std):
        return torch.empty(shape, dtype=torch.bfloat16, device="cuda").normal_(
            0.0, std, generator=g).cpu()

    w = {"embed": init((mc.vocab_size, d), 0.02), "lm_head": init((mc.vocab_size, d), 0.02),
         "final_norm": torch.ones(d, dtype=torch.bfloat16), "layers": []}
    std_o = 0.02 / math.sqrt(2 * mc.num_layers)
    for _ in range(mc.num_layers):
        w["layers"].append({
            "in_norm": torch.ones(d, dtype=torch.bfloat16),
            "post_norm": torch.ones(d, dtype=torch.bfloat16),
            "qkv": init(((mc.num_heads + 2 * mc.num_kv_heads) * D, d), 0.02),
            "o": init((d, mc.num_heads * D), std_o),
            "gate_up": init((2 * mc.intermediate_size, d), 0.02),
            "down": init((d, mc.intermediate_size), std_o)})
    return w


def to_f32(w):
    if isinstance(w, dict):
        return {k: to_f32(v) for k, v in w.items()}
    if isinstance(w, list):
        return [to_f32(v) for v in w]
    return w.float() if isinstance(w, torch.Tensor) else w


def swapped_kv_head(w32: dict, mc) -> dict:
    """Negative control: layer 0's first two kv heads exchanged."""
    bad = dict(w32)
    bad["layers"] = [dict(x) for x in w32["layers"]]
    D, hq = mc.head_dim, mc.num_heads
    qkv = bad["layers"][0]["qkv"].clone()
    k0 = hq * D
    qkv[k0:k0 + D], qkv[k0 + D:k0 + 2 * D] = qkv[k0 + D:k0 + 2 * D].clone(), \
        qkv[k0:k0 + D].clone()
    bad["layers"][0]["qkv"] = qkv
    return bad


def check_tap(tap_dir: str, mc, w32: dict, rel_tol: float = 0.05) -> tuple[float, float, int]:
    """(fraction of rows within ``rel_tol`` of the oracle, worst error, rows)
    over every sequence the pods serving model ``mc.name`` dumped."""
    from omnia_amd.ops import reference as ref

    files = sorted(glob.glob(os.path.join(tap_dir, f"seq-{mc.name}-*.pt")))
    assert files, f"the pod dumped no logit rows into {tap_dir}"
    ok = total = 0
    worst = 0.0
    for f in files:
        d = torch.load(f, weights_only=True)
        prompt, output, rows = d["prompt"], d["output"], d["rows"]
        assert len(output) <= rows.shape[0] <= len(output) + 1, (f, rows.shape, len(output))
        want = ref.dense_forward(mc, w32, (prompt + output)[:-1])[len(prompt) - 1:]
        for g, r in zip(rows[:len(output)], want):
            err = float((g - r).abs().max() / r.abs().max())
            worst = max(worst, err)
            ok += err < rel_tol
            total += 1
    return ok / max(1, total), worst, total
