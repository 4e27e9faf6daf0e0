"""Data-path parity: prompt template, prompt-token masking, pad collator and
the map / filter / shuffle(42) pipeline of hdpissa_amd.data against the reference's own functions
(hp:24-28, 158-210, 243-261) run on the same inputs with the same deterministic stub tokenizer
(tests/golden/make_golden.py gen_data -> data_path.npz).  CPU only."""
import os

import numpy as np
import torch

from helpers import StubTokenizer, synthetic_instructions

GOLDEN = os.path.join(os.path.dirname(os.path.abspath(__file__)), "golden")


def _unragged(z, prefix):
    flat, lens = z[f"{prefix}_flat"], z[f"{prefix}_len"]
    out, o = [], 0
    for n in lens:
        out.append(flat[o:o + n].tolist())
        o += n
    return out


def test_tokenize_and_mask_match_reference():
    from hdpissa_amd import data
    z = np.load(os.path.join(GOLDEN, "data_path.npz"))
    tok = StubTokenizer(model_max_length=int(z["model_max_length"]))
    ex = {"query": z["query"].tolist(), "response": z["response"].tolist()}
    assert ex == synthetic_instructions(20, 7)
    out = data.train_tokenize_function(ex, tok, "query", "response")
    assert out["input_ids"] == _unragged(z, "input_ids")
    assert out["labels"] == _unragged(z, "labels")
    # rows truncated before their response carry no supervised token and are dropped (hp:255-260)
    dropped = [i for i, lab in enumerate(out["labels"]) if not data.has_valid_labels({"labels": lab})]
    assert dropped and all(len(out["input_ids"][i]) == tok.model_max_length for i in dropped)


def test_collator_matches_reference():
    from hdpissa_amd import data
    z = np.load(os.path.join(GOLDEN, "data_path.npz"))
    tok = StubTokenizer(model_max_length=int(z["model_max_length"]))
    ids, labs = _unragged(z, "input_ids"), _unragged(z, "labels")
    got = data.DataCollatorForSupervisedDataset(tok)([{"input_ids": ids[i], "labels": labs[i]} for i in range(4)])
    for k in ("input_ids", "labels", "attention_mask"):
        assert np.array_equal(got[k].numpy(), z[f"collated_{k}"]), k
    # pad = eos (hp:226-227): the mask also drops each row's final eos, as in the reference
    assert got["attention_mask"].dtype == torch.bool


def test_dataset_pipeline_matches_reference():
    import datasets
    from hdpissa_amd import data
    z = np.load(os.path.join(GOLDEN, "data_path.npz"))
    tok = StubTokenizer(model_max_length=int(z["model_max_length"]))
    raw = datasets.Dataset.from_dict({"query": z["query"].tolist(), "response": z["response"].tolist()})
    ds = data.build_train_dataset(raw, tok, "query", "response")
    assert [list(r) for r in ds["input_ids"]] == _unragged(z, "pipeline_input_ids")


def test_dataloader_shards_are_disjoint_and_drop_last():
    import datasets
    from hdpissa_amd import data
    tok = StubTokenizer()
    raw = datasets.Dataset.from_dict(synthetic_instructions(40, 3))
    ds = data.build_train_dataset(raw, tok, "query", "response")
    seen = []
    for rank in range(2):
        dl = data.make_dataloader(ds, tok, batch_size=3, world_size=2, rank=rank)
        rows = 0
        for b in dl:
            assert b["input_ids"].shape == b["labels"].shape == b["attention_mask"].shape
            assert b["input_ids"].shape[0] == 3
            rows += 3
            seen.extend(tuple(r[m].tolist()) for r, m in zip(b["input_ids"], b["attention_mask"]))
        assert rows == (len(ds) // 2) // 3 * 3   # DistributedSampler shard, drop_last batches
    assert len(seen) == len(set(seen))
