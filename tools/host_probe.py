"""Host time per XL bs120 training step (no synchronisation inside the loop) against the device time
per step: if the host needs about as long as the GPU, launch overhead bounds the step."""
import os
import sys
import time

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, REPO)
sys.path.insert(0, os.path.join(REPO, "sdp-net_amd"))
import torch  # noqa: E402
import bench  # noqa: E402
import model as sdp  # noqa: E402
import sdpnet_train  # noqa: E402

dev = torch.device("cuda")
torch.manual_seed(0)
m = sdp.MainModel.from_dict(**bench.XL_CFG).to(dev).train()
opt = sdpnet_train.AdamW(m.parameters(), lr=0.0015, weight_decay=0.05)
B = int(os.environ.get("B", "120"))
x = torch.randn(B, 3, 224, 224, device=dev)
y = torch.randint(0, 1000, (B,), device=dev)


def step():
    opt.zero_grad(set_to_none=True)
    with torch.autocast("cuda", dtype=torch.bfloat16):
        loss = sdpnet_train.cross_entropy(m(x), y, 0.1)
    opt.scale(loss).backward()
    opt.step(grad_scale=None, max_norm=5.0)


for _ in range(3):
    step()
torch.cuda.synchronize()
hs = []
t0 = time.perf_counter()
for _ in range(10):
    a = time.perf_counter()
    step()
    hs.append(time.perf_counter() - a)
t_host = time.perf_counter() - t0
torch.cuda.synchronize()
t_all = time.perf_counter() - t0
print(f"B {B}: host per step {1e3 * t_host / 10:.1f} ms (steps: {' '.join(f'{1e3 * h:.1f}' for h in hs)}), "
      f"wall per step incl. drain {1e3 * t_all / 10:.1f} ms")
import cProfile, pstats, io  # noqa: E402,E401
pr = cProfile.Profile()
pr.enable()
step()
pr.disable()
torch.cuda.synchronize()
s = io.StringIO()
pstats.Stats(pr, stream=s).sort_stats("tottime").print_stats(25)
print(s.getvalue()[:6000])
