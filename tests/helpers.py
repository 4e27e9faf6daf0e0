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


class StubTokenizer:
    """Deterministic byte-level tokenizer with the HF call surface the reference's data path
    uses (hp:158-210, 220-227): __call__(text, max_length=, truncation=) -> .input_ids, plus
    eos_token, pad_token_id (= eos, as hp:226-227 sets it when the tokenizer has none) and
    model_max_length.  bos = 1, eos = 2, bytes -> 3 + (b % 250): ids < 256.  TEST INFRASTRUCTURE."""
    eos_token = "</s>"
    eos_token_id = 2
    bos_token_id = 1

    def __init__(self, model_max_length=200):
        self.model_max_length = model_max_length
        self.pad_token_id = self.eos_token_id

    def __call__(self, text, max_length=None, truncation=False):
        import types
        ids = [self.bos_token_id]
        for i, part in enumerate(text.split(self.eos_token)):
            if i:
                ids.append(self.eos_token_id)
            ids.extend(3 + (b % 250) for b in part.encode())
        if truncation and max_length is not None:
            ids = ids[:max_length]
        return types.SimpleNamespace(input_ids=ids)


def synthetic_instructions(n, seed):
    """n (instruction, response) pairs of varied lengths; every 5th prompt is long enough to be
    truncated past the response (its labels end up all -100 and the row is filtered)."""
    g = np.random.default_rng(seed)
    words = ["add", "the", "numbers", "what", "is", "sum", "of", "x", "y", "solve", "for", "prove", "that", "tokens",
             "matrix", "rank", "slice", "update", "gpu", "cache"]
    qs, rs = [], []
    for i in range(n):
        nq = int(g.integers(2, 8)) + (40 if i % 5 == 4 else 0)
        nr = int(g.integers(1, 6))
        qs.append(" ".join(words[int(k)] for k in g.integers(0, len(words), nq)))
        rs.append(" ".join(words[int(k)] for k in g.integers(0, len(words), nr)))
    return {"query": qs, "response": rs}


QWEN_TINY = dict(vocab_size=256, hidden_size=64, intermediate_size=128, num_hidden_layers=2, num_attention_heads=4,
                 num_key_value_heads=2, max_position_embeddings=256)
QWEN_TARGETS = ["q_proj", "o_proj", "k_proj", "v_proj", "gate_proj", "up_proj", "down_proj"]

# Qwen2.5-0.5B architecture (BASELINE configs[0]; hp:444's default model), random-initialised
QWEN_05B = dict(vocab_size=151936, hidden_size=896, intermediate_size=4864, num_hidden_layers=24,
                num_attention_heads=14, num_key_value_heads=2, max_position_embeddings=32768, rope_theta=1000000.0,
                tie_word_embeddings=True, rms_norm_eps=1e-6)


def model_checksums(model):
    """A few float64 sums over the parameters: a reconstructed model (same seed, same image)
    must reproduce them exactly before a trajectory is compared."""
    out = []
    for n, p in sorted(model.named_parameters())[:12]:
        t = p.detach().cpu().numpy().astype(np.float64).ravel()  # numpy's pairwise sum: thread-count independent
        out.extend([float(np.sum(t)), float(np.sum(t * t))])
    return out
