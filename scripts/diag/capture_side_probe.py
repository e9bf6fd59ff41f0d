"""Step by step: an eager key-split call on a fresh side stream while the default capture stream records
a graph (global mode). Prints the caching allocator's segment count around each step and which step
raises (diagnostic for tests/test_gpu_parity.py::test_first_key_split_call_beside_a_graph_capture)."""
import sys

import torch

sys.path.insert(0, ".")
import flash_attention_cute_amd as m  # noqa: E402
from flash_attention_cute_amd import _debug  # noqa: E402

dev = torch.device("cuda:0")
g0 = torch.Generator().manual_seed(41)
q, k, v = (torch.randn(1, h, 1024, 128, generator=g0).half().to(dev) for h in (4, 2, 2))
_debug.set_split(2)
eager = m.flash_attn_func(q, k, v, causal=True)
side = torch.cuda.Stream()
seg = lambda: torch.cuda.memory_stats().get("segment.all.allocated", 0)  # noqa: E731
mode = sys.argv[1] if len(sys.argv) > 1 else "warm"
if mode == "warm":
    with torch.cuda.stream(side):
        warm = [torch.empty(64 << 20, dtype=torch.uint8, device=dev), torch.empty(4096, dtype=torch.uint8, device=dev)]
        del warm
torch.cuda.synchronize()
print("segments before capture", seg(), flush=True)
g = torch.cuda.CUDAGraph()
steps = []
try:
    with torch.cuda.graph(g):
        out = m.flash_attn_func(q, k, v, causal=True)
        steps.append(("captured op", seg()))
        with torch.cuda.stream(side):
            a = torch.empty_like(q)
            steps.append(("side empty_like", seg()))
            w = torch.empty(3 << 20, dtype=torch.uint8, device=dev)
            steps.append(("side ws-sized empty", seg()))
            del a, w
            try:
                side_out = m.flash_attn_func(q, k, v, causal=True)
                steps.append(("side op", seg(), _debug.last_layout()))
            except Exception as e:  # noqa: BLE001
                steps.append(("side op FAILED", str(e).splitlines()[0]))
                raise
except Exception as e:  # noqa: BLE001
    steps.append(("capture FAILED", str(e).splitlines()[0]))
for s in steps:
    print(s, flush=True)
