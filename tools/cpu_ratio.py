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


def rate(f, reps=2):
    t0 = time.perf_counter()
    for _ in range(reps):
        f()
    return 16 * reps / (time.perf_counter() - t0)


# interleaved rounds (the two sides alternate, so drift in clock / load hits both), median ratio
rounds = int(os.environ.get("ROUNDS", "5"))
with torch.no_grad():
    m(x)
    orc.forward(x, sd, cfg)
    rr, ro = [], []
    for _ in range(rounds):
        rr.append(rate(lambda: m(x)))
        ro.append(rate(lambda: orc.forward(x, sd, cfg)))
ratios = sorted(o / r for o, r in zip(ro, rr))
med = ratios[len(ratios) // 2]
print(f"threads {torch.get_num_threads()}: reference {sorted(rr)[len(rr) // 2]:.2f} img/s, "
      f"oracle {sorted(ro)[len(ro) // 2]:.2f} img/s, oracle/reference median {med:.3f} "
      f"(range {ratios[0]:.3f}-{ratios[-1]:.3f} over {rounds} interleaved rounds)")
if len(sys.argv) > 1:  # write the record bench.py attaches to cpu_baseline
    import json
    json.dump({"port_vs_reference": round(med, 3), "range": [round(ratios[0], 3), round(ratios[-1], 3)],
               "rounds": rounds, "threads": torch.get_num_threads(),
               "workload": "SdP-Net-M fp32 eval forward, batch 16, 224x224, same weights and inputs",
               "measured": time.strftime("%Y-%m-%d"), "where": "build container (the reference is not on the GPU box)",
               "reference_img_s": round(sorted(rr)[len(rr) // 2], 3), "oracle_img_s": round(sorted(ro)[len(ro) // 2], 3)},
              open(sys.argv[1], "w"), indent=1)
