"""The data path in front of the hot path: instruction prompts -> token ids / masked labels ->
padded micro-batches on each rank's shard (hp:24-28, 158-210, 243-277).

Host-side and format-only (no kernels): the tokenizer, ``datasets`` and the DataLoader are the
same libraries the reference drives, so a user of the reference gets identical micro-batches.
Contract kept from the reference:
  * the Alpaca-style prompt template (hp:24-28) around each instruction; the target is the
    response + "\\n" + eos (hp:206-210);
  * prompt tokens of every label row are -100 (hp:171-184): loss on the response only;
    rows whose labels are all -100 (prompt truncated past max_length) are dropped (hp:255-260);
  * right padding to the longest sample of the micro-batch, pad id in input_ids, -100 in labels,
    attention_mask = input_ids != pad (hp:186-204) -- when the tokenizer has no pad token the
    reference sets pad = eos (hp:226-227), so the mask also drops each sample's final eos;
  * one shuffle with seed 42, then a non-shuffling DistributedSampler shard per rank and
    drop_last batches (hp:261-277).
"""
from __future__ import annotations

import copy
from typing import Dict, List, Sequence

import torch

PROMPT = (
    "Below is an instruction that describes a task. "
    "Write a response that appropriately completes the request.\n\n"
    "### Instruction:\n{instruction}\n\n### Response:"
)


def tokenize_strings(strings: Sequence[str], tokenizer) -> Dict[str, list]:
    """hp:158-169: each string tokenized on its own, truncated to tokenizer.model_max_length."""
    ids = [list(tokenizer(s, max_length=tokenizer.model_max_length, truncation=True).input_ids) for s in strings]
    lens = [len(x) for x in ids]
    return dict(input_ids=ids, labels=ids, input_ids_lens=lens, labels_lens=lens)


def preprocess(sources: Sequence[str], targets: Sequence[str], tokenizer) -> Dict[str, list]:
    """hp:171-184: tokenize prompt + response, and mask the prompt's tokens out of the labels."""
    full = tokenize_strings([s + t for s, t in zip(sources, targets)], tokenizer)
    prompt_lens = tokenize_strings(sources, tokenizer)["input_ids_lens"]
    labels = copy.deepcopy(full["input_ids"])
    for row, n in zip(labels, prompt_lens):
        row[:n] = [-100] * len(row[:n])
    return dict(input_ids=full["input_ids"], labels=labels)


def train_tokenize_function(examples, tokenizer, query: str, response: str) -> Dict[str, list]:
    """hp:206-210 (a ``datasets.map`` batch function)."""
    sources = [PROMPT.format_map({"instruction": q}) for q in examples[query]]
    targets = [f"{a}\n{tokenizer.eos_token}" for a in examples[response]]
    return preprocess(sources, targets, tokenizer)


def has_valid_labels(example) -> bool:
    """hp:255-257: keep rows with at least one supervised token."""
    return any(lab != -100 for lab in example["labels"])


class DataCollatorForSupervisedDataset:
    """hp:186-204: right-pad a list of examples to the longest one."""

    def __init__(self, tokenizer):
        self.tokenizer = tokenizer

    def __call__(self, instances: Sequence[Dict]) -> Dict[str, torch.Tensor]:
        pad = self.tokenizer.pad_token_id
        ids = [torch.as_tensor(x["input_ids"]) for x in instances]
        labs = [torch.as_tensor(x["labels"]) for x in instances]
        input_ids = torch.nn.utils.rnn.pad_sequence(ids, batch_first=True, padding_value=pad)
        labels = torch.nn.utils.rnn.pad_sequence(labs, batch_first=True, padding_value=-100)
        return dict(input_ids=input_ids, labels=labels, attention_mask=input_ids.ne(pad))


def build_train_dataset(raw_dataset, tokenizer, query: str, response: str, num_proc=None, seed: int = 42):
    """hp:243-261: tokenize (batched map), drop rows without supervised tokens, shuffle once."""
    ds = raw_dataset.map(train_tokenize_function, batched=True, batch_size=3000, num_proc=num_proc,
                         remove_columns=raw_dataset.column_names, fn_kwargs=dict(tokenizer=tokenizer, query=query,
                                                                                  response=response))
    return ds.filter(has_valid_labels).shuffle(seed=seed)


def make_dataloader(dataset, tokenizer, batch_size: int, world_size: int, rank: int, num_workers: int = 0,
                    pin_memory: bool = False):
    """hp:263-277: this rank's shard (DistributedSampler, no shuffle), drop_last micro-batches."""
    from torch.utils.data import DataLoader
    from torch.utils.data.distributed import DistributedSampler
    sampler = DistributedSampler(dataset, num_replicas=world_size, rank=rank, shuffle=False)
    return DataLoader(dataset, drop_last=True, batch_size=batch_size, sampler=sampler, num_workers=num_workers,
                      pin_memory=pin_memory, collate_fn=DataCollatorForSupervisedDataset(tokenizer))


def micro_batch_rows(batches: List[Dict[str, torch.Tensor]]) -> List[int]:
    """Padded rows (batch x longest sample) of each micro-batch: the T the probe kernels see."""
    return [int(b["input_ids"].numel()) for b in batches]
