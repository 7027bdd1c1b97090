"""Print the A/B runs of scripts/ab_scale.sh (gpurun_out/abs_<i>.jsonl/.log)."""
import glob
import json
import re

for p in sorted(glob.glob("gpurun_out/abs_*.jsonl"), key=lambda x: int(re.findall(r"\d+", x)[-1])):
    try:
        d = json.loads(open(p).readline())
    except (ValueError, OSError):
        print(p, "no line")
        continue
    print(p, d["env"], "T", d["timesteps"], "gpu s", d["gpu_end_to_end_s"], "bit-exact prefix", d["prefix_bit_exact"])
    print("   sections", [round(x, 1) for x in d["plan_section_ms"]], "waits", round(d["coop_wait_ms"], 1))
    for ln in open(p.replace(".jsonl", ".log")):
        if ln.startswith("[k_plan]") and ("backlog" in ln or "worker A*" in ln):
            print("  ", ln.strip()[:200])
