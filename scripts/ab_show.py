"""Print the A/B runs of scripts/ab_plan.sh (gpurun_out/ab_<i>.json/.err)."""
import glob
import json
import re

for p in sorted(glob.glob("gpurun_out/ab_*.json"), key=lambda x: int(re.findall(r"\d+", x)[-1])):
    try:
        d = json.load(open(p))
    except ValueError:
        print(p, "no line")
        continue
    k = d["kernel_stats"]
    print(p, d["ms_per_step"], "ms/plan", "T", d["config"]["timesteps_per_plan"])
    print("   sections", [round(x / 2, 1) for x in k["plan_section_ms"]])
    print("   waits   ", [round(x / 2, 1) for x in k["coop_wait_sec_ms"]], [x // 2 for x in k["coop_waits_sec"]])
    for ln in open(p.replace(".json", ".err")):
        if ln.startswith("[k_plan]"):
            print("  ", ln.strip()[:220])
