"""One-screen summary of bench.py JSON lines in log files: step time, parity, per-class ms/step.
    python tools/bench_summary.py gpurun_out/bench.log [...]"""
import json
import sys

for path in sys.argv[1:]:
    for line in open(path):
        line = line.strip()
        if not line.startswith("{"):
            continue
        b = json.loads(line)
        par = b.get("parity") or {}
        print(f"{path}: {b['config'].get('workload', '')[:3]} {b['ms_per_step']:.1f} ms/step "
              f"value {b['value']:.4g} parity {par.get('ok')} ({par.get('iterations_pinned')} it)")
        rl = b.get("roofline") or {}
        ks = sorted(rl.get("kernels", []), key=lambda k: -k["ms_per_step"])
        print("   " + "  ".join(f"{k['class']} {k['ms_per_step']:.1f}" for k in ks))
        ph = b.get("phases_ms_per_step") or {}
        print("   phases: " + "  ".join(f"{k} {v:.1f}" for k, v in ph.items() if v))
