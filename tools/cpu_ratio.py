"""Container-only: speed of the CPU oracle (oracle/sdpnet_oracle.py, bench.py's cpu_baseline leg)
against the reference's own CPU forward (imported from /root/reference with a wandb stub) on
the same weights and inputs: SdP-Net-M eval fp32, batch 16, this machine's threads.  Records the
ratio that qualifies bench.py's cpu_baseline (kind "port")."""
import os
import sys
import time
import types

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [os.path.join(REPO, "oracle"), os.path.join(REPO, "tests", "golden")]
sys.dont_write_bytecode = True
import torch  # noqa: E402
import sdpnet_oracle as orc  # noqa: E402
import synth  # noqa: E402

sys.modules.setdefault("wandb", types.ModuleType("wandb"))
sys.path.insert(0, "/root/reference")
import model as ref_model  # noqa: E402

torch.set_num_threads(len(os.sched_getaffinity(0)))
cfg = synth.canonical("M")
torch.manual_seed(0)
m = ref_model.MainModel.from_dict(**cfg).eval()
sd = synth.synth_state_dict(m, 231424314)
m.load_state_dict(sd)
x = synth.synth_images(0, 16, 224)


def rate(f, reps=3):
    f()
    t0 = time.perf_counter()
    for _ in range(reps):
        f()
    return 16 * reps / (time.perf_counter() - t0)


with torch.no_grad():
    r_ref = rate(lambda: m(x))
    r_orc = rate(lambda: orc.forward(x, sd, cfg))
print(f"threads {torch.get_num_threads()}: reference {r_ref:.2f} img/s, oracle {r_orc:.2f} img/s, "
      f"oracle/reference {r_orc / r_ref:.3f}")
