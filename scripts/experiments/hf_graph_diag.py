#!/usr/bin/env python3
"""Diagnose tests/test_hf_patch.py::test_patched_llama_static_cache_decode_steps_replay_one_hip_graph:
token ids of (ref) unpatched static-cache generate, (eager) the step loop run eagerly, (graph) the
same loop replaying one captured HIP graph -- each patched and unpatched."""
import sys
import warnings
from pathlib import Path

import torch

ROOT = Path(__file__).resolve().parents[2]
sys.path.insert(0, str(ROOT))
sys.path.insert(0, str(ROOT / "tests"))
from transformers import StaticCache  # noqa: E402
from transformers.models.llama import modeling_llama as ml  # noqa: E402

import test_hf_patch as T  # noqa: E402
from flash_attention_cute_amd import hf_attention  # noqa: E402

dev = "cuda:0"
model, ids, mask = T.tiny_generator(dev, True)
model = model.half()
n_new = 24
with torch.no_grad():
    ref = model.generate(ids, attention_mask=mask, max_new_tokens=n_new, do_sample=False, pad_token_id=0,
                         cache_implementation="static")
b, n0 = ids.shape
total = n0 + n_new


def loop(patch, graph_mode):
    cache = StaticCache(config=model.config, max_cache_len=total)
    full = torch.zeros(b, total, dtype=torch.long, device=dev)
    full[:, :n0] = mask
    pid = (mask.long().cumsum(1) - 1).clamp(min=0)
    toks = []
    ctx = T.patched(ml.LlamaAttention) if patch else T._null()
    with torch.no_grad(), warnings.catch_warnings(), ctx:
        warnings.simplefilter("ignore")
        out = model(ids, attention_mask=full[:, :n0], position_ids=pid, past_key_values=cache, use_cache=True,
                    cache_position=torch.arange(n0, device=dev))
        toks.append(out.logits[:, -1].argmax(-1, keepdim=True))
        tok_buf, pos_buf = toks[-1].clone(), pid[:, -1:] + 1
        slot = torch.tensor([n0], device=dev)
        full[:, n0] = 1

        def step():
            return model(tok_buf, attention_mask=full, position_ids=pos_buf, past_key_values=cache, use_cache=True,
                         cache_position=slot).logits[:, -1]

        def advance(lg, i):
            toks.append(lg.argmax(-1, keepdim=True))
            tok_buf.copy_(toks[-1])
            full[:, n0 + i] = 1
            pos_buf.add_(1)
            slot.add_(1)

        advance(step(), 1)
        torch.cuda.synchronize()
        if graph_mode:
            g = torch.cuda.CUDAGraph()
            with torch.cuda.graph(g):
                lb = step()
            for i in range(2, n_new):
                g.replay()
                advance(lb, i)
        else:
            for i in range(2, n_new):
                advance(step(), i)
        torch.cuda.synchronize()
    return torch.cat(toks, dim=1)


print("ref  ", ref[:, n0:].tolist(), flush=True)
for patch in (False, True):
    for gm in (False, True):
        try:
            got = loop(patch, gm)
            bad = (got != ref[:, n0:]).nonzero().tolist()
            print(f"patch={patch} graph={gm}: first mismatches {bad[:4]} errors={hf_attention.mask_errors(dev)}",
                  got.tolist(), flush=True)
        except Exception as e:  # noqa: BLE001
            print(f"patch={patch} graph={gm}: {type(e).__name__}: {str(e)[:300]}", flush=True)
