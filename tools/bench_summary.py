"""One-line summary of a bench.py JSON line (tools/gpu.sh).  usage: python tools/bench_summary.py FILE"""
import json
import sys

d = json.loads([x for x in open(sys.argv[1]).read().splitlines() if x.startswith("{")][-1])
r = d["roofline"]
parts = [f"cfg5 {d['value']} GiB/s", f"{d['ms_per_step']} ms/step", f"frac {r['frac']}",
         f"traffic/alg {r.get('traffic_over_alg')}"]
for k in ("blockhash", "emit"):
    if k in d.get("kernel_rooflines", {}):
        kr = d["kernel_rooflines"][k]
        parts.append(f"{k} {kr['avg_launch_ms']} ms ({kr['frac']})")
if "live_cache" in d:
    lv = d["live_cache"]
    parts.append(f"live {lv['value']} GiB/s ({lv['vs_headline']} of headline, replay "
                 f"{lv['window_replay']['host_ms_per_run']} ms/run)")
oc = d.get("other_configs", {})
for k in ("cfg2", "cfg3"):
    if k in oc:
        parts.append(f"{k} {oc[k]['value']}")
if "decode" in d:
    parts.append(f"dec {d['decode']['value']} ({d['decode']['roofline']['frac']})")
if "e2e_host_gibs" in d:
    parts.append(f"e2e {d['e2e_host_gibs']}")
if d.get("cpu_baseline"):
    parts.append(f"cpu {d['cpu_baseline']['value']} ({d['cpu_baseline']['cores']} cores)")
print(" | ".join(parts))
print("kernels", d.get("kernel_ms_per_step"))
