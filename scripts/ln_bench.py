"""LayerNorm microbenchmark on the CLIP shape (32896 x 1280 f32 -> bf16): time, TB/s, error vs torch."""
import sys, torch
sys.path.insert(0, '.')
from boxfusion_amd import _lib
x = torch.randn(32896, 1280, device="cuda") * 3 + 1
g = torch.randn(1280, device="cuda"); b = torch.randn(1280, device="cuda")
out = torch.empty(32896, 1280, device="cuda", dtype=torch.bfloat16)
for _ in range(3): _lib.layernorm(x, g, b, 1e-5, out=out)
torch.cuda.synchronize()
s, e = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
best = 1e9
for r in range(5):
    s.record()
    for _ in range(20): _lib.layernorm(x, g, b, 1e-5, out=out)
    e.record(); torch.cuda.synchronize(); best = min(best, s.elapsed_time(e) / 20)
ref = torch.nn.functional.layer_norm(x, (1280,), g, b, 1e-5)
print(f"layernorm 32896x1280: {best*1e3:.1f} us, {252.6e6/(best*1e-3)/1e12:.2f} TB/s, err {((out.float()-ref).norm()/ref.norm()).item():.1e}")
