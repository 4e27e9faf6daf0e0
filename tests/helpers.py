"""Shared test builders (models shaped like the golden step fixtures)."""
import numpy as np
import torch
import torch.nn as nn

STEP_SPECS = {
    "f32_tall": [("layers.0.q_proj", 64, 48, True)],
    "f32_wide": [("layers.0.down_proj", 40, 72, False)],
    "bf16_tall": [("layers.0.q_proj", 64, 48, True)],
    "f32_two": [("layers.0.q_proj", 48, 48, False), ("layers.1.up_proj", 64, 32, False)],
}


class Box(nn.Module):
    pass


def wkey(W: torch.Tensor):
    return (tuple(W.shape), round(float(W.float().double().sum().item()), 6))


def build_fixture_model(z, case, device="cpu"):
    """Container with the fixture's modules (layers.<i>.<proj>) and a factor table holding
    EVERY rank's reference factors: {wkey(W): (A_all [Wn*r, in], B_all [Wn, out, r])}."""
    specs = STEP_SPECS[case]
    dt = torch.bfloat16 if str(z["dtype"]) == "bfloat16" else torch.float32
    wn = int(z["world_size"])
    root = Box()
    root.layers = nn.ModuleList()
    table = {}
    for j, (name, out, inn, has_bias) in enumerate(specs):
        idx = int(name.split(".")[1])
        while len(root.layers) <= idx:
            root.layers.append(Box())
        lin = nn.Linear(inn, out, bias=has_bias)
        with torch.no_grad():
            lin.weight.copy_(torch.from_numpy(z[f"r0.{j}.W0"]))
        lin = lin.to(device=device, dtype=dt)
        for p in lin.parameters():
            p.requires_grad = False
        setattr(root.layers[idx], name.split(".")[-1], lin)
        A_all = torch.cat([torch.from_numpy(z[f"r{i}.{j}.A"]) for i in range(wn)]).to(device)
        B_all = torch.stack([torch.from_numpy(z[f"r{i}.{j}.B"]) for i in range(wn)]).to(device)
        table[wkey(lin.weight)] = (A_all, B_all)
    return root, table, [s[0].split(".")[-1] for s in specs], dt


def rel_err(x, ref):
    x = np.asarray(x, np.float64)
    ref = np.asarray(ref, np.float64)
    d = np.linalg.norm(ref)
    return float(np.linalg.norm(x - ref) / (d if d > 0 else 1.0))
