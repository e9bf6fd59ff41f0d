"""GPU helper: pick a seed for tests/test_hf_patch.py's greedy-generate test -- the fp32 greedy
trajectory's smallest top-2 logit margin on THIS device, and whether unpatched HF fp16 reproduces the
fp32 token ids (dense and left-padded prompts)."""
import sys
import warnings

import torch
import transformers

sys.path.insert(0, ".")
from tests.test_hf_patch import greedy_margins, tiny_llama  # noqa: E402

warnings.simplefilter("ignore")
dev = torch.device("cuda:0")
for ir in (0.1, 0.2, 0.3):
    for seed in range(12):
        row = []
        for padded in (False, True):
            cfg = tiny_llama(hq=8, hkv=2, d=128, layers=2)
            cfg.initializer_range = ir
            torch.manual_seed(seed)
            model = transformers.LlamaForCausalLM(cfg).to(dev).eval()
            ids = torch.randint(0, cfg.vocab_size, (2, 48), device=dev)
            mask = torch.ones_like(ids)
            if padded:
                mask[1, :17] = 0
                ids[1, :17] = 0
            kw = dict(attention_mask=mask, max_new_tokens=24, do_sample=False, pad_token_id=0)
            with torch.no_grad():
                r32 = model.generate(ids, **kw)
                m = greedy_margins(model, r32, 48, mask).min().item()
                r16 = model.half().generate(ids, **kw)
            row.append((round(m, 3), bool(torch.equal(r16, r32)), len(set(r32[:, 48:].flatten().tolist()))))
        print(ir, seed, row, flush=True)
