#!/bin/bash
# VALU issue ceiling on the GPU box (tools/microbench/myers_ilp.hip): independent v_bitop3 chains
# and the 64-bit Myers step at 1..8 waves per SIMD, with the shader clock sampled before and after.
# Usage: tools/microbench/run_ceiling.sh OUT.json
set -e -o pipefail
here=$(dirname "$0")
out=$1
/opt/rocm/bin/hipcc -Wno-unused-value -O3 -std=c++17 --offload-arch=gfx950 -o /tmp/myers_ilp "$here/myers_ilp.hip"
clk0=$(timeout -k 5 30 rocm-smi --showclocks 2>/dev/null | grep -i "sclk" | head -2 | tr '\n' ' ' || true)
res=$(timeout -k 10 120 /tmp/myers_ilp)
clk1=$(timeout -k 5 30 rocm-smi --showclocks 2>/dev/null | grep -i "sclk" | head -2 | tr '\n' ' ' || true)
python3 - "$out" "$clk0" "$clk1" <<PY
import json, re, sys
res = """$res"""
lines = [l for l in res.splitlines() if l.strip()]
m = re.search(r"\nbitop3 chain x4: ([0-9.]+) ms\s+([0-9.]+) T lane-ops/s", "\n" + res)
mi = re.search(r"bitop3 independent x8: ([0-9.]+) ms\s+([0-9.]+) T lane-ops/s", res)
ms_ = re.search(r"stamped bitop3 chain x4 after ([0-9.]+) ms / (\d+) launches: ([0-9.]+) ms\s+"
                r"([0-9.]+) T lane-ops/s\s+clock ([0-9.]+) MHz \(median of (\d+) blocks, p10 "
                r"([0-9.]+) p90 ([0-9.]+)\)", res)
steps = [dict(chains=int(a), waves_per_simd=int(b), ms=float(c), g_lane_steps_per_s=float(d))
         for a, b, c, d in re.findall(r"chains (\d+) waves/SIMD (\d+): ([0-9.]+) ms\s+([0-9.]+) G", res)]
out = {"what": "VALU issue ceiling, gfx950 (MI355X): v_bitop3 dependency chains x4 per lane at "
               "8192 x 256 threads; 64-bit Myers step (myers_step_hw) by chains per lane and waves "
               "per SIMD", "source": "tools/microbench/myers_ilp.hip",
       "bitop3_t_lane_ops_per_s": float(m.group(2)) if m else None,
       "bitop3_dependent_chain_t_lane_ops_per_s": float(m.group(2)) if m else None,
       "bitop3_independent_t_lane_ops_per_s": float(mi.group(2)) if mi else None,
       "nominal_t_lane_ops_per_s": 256 * 4 * 32 * 2.4e9 / 1e12,
       "stamped": (dict(warm_ms=float(ms_.group(1)), warm_launches=int(ms_.group(2)),
                        ms=float(ms_.group(3)), t_lane_ops_per_s=float(ms_.group(4)),
                        clock_mhz=float(ms_.group(5)), blocks=int(ms_.group(6)),
                        clock_mhz_p10=float(ms_.group(7)), clock_mhz_p90=float(ms_.group(8)),
                        peak_t_lane_ops_per_s_at_clock=256 * 4 * 32 * float(ms_.group(5)) * 1e6 / 1e12,
                        frac_of_peak_at_clock=float(ms_.group(4)) /
                        (256 * 4 * 32 * float(ms_.group(5)) * 1e6 / 1e12),
                        how="s_memtime / s_memrealtime x 100 MHz around the loop, first lane of "
                            "every block, after >= 2 s of back-to-back launches (MI355X_MICROARCH.md "
                            "DVFS item 6); stamps in their own buffer")
                   if ms_ else None),
       "myers_step": steps,
       "best_g_lane_steps_per_s": max((s["g_lane_steps_per_s"] for s in steps), default=None),
       "sclk_before": sys.argv[2], "sclk_after": sys.argv[3], "raw": lines}
json.dump(out, open(sys.argv[1], "w"), indent=1)
print(json.dumps({k: out[k] for k in ("bitop3_t_lane_ops_per_s", "best_g_lane_steps_per_s", "stamped")}))
PY
