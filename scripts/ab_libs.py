"""Cross-process A/B of two builds of the library (compile-flag experiments).
usage: python scripts/_ab_libs.py libA.so libB.so [bench args]"""
import json, subprocess, sys
libs = [a for a in sys.argv[1:] if a.endswith(".so")]
extra = [a for a in sys.argv[1:] if not a.endswith(".so")]
code = ("import sys; sys.path.insert(0,'.'); from pathlib import Path; import dexiraft_amd; "
        "dexiraft_amd._native.LIB_PATH = Path(sys.argv[1]); sys.argv = ['bench.py'] + sys.argv[2:]; "
        "import runpy; runpy.run_path('bench.py', run_name='__main__')")
res = {l: [] for l in libs}
for rnd in range(3):
    for l in libs:
        out = subprocess.run([sys.executable, "-c", code, l, "--steps", "30", "--warmup", "3",
                              "--no-cpu-baseline", *extra], capture_output=True, text=True, timeout=300)
        line = [x for x in out.stdout.splitlines() if x.startswith("{")][-1]
        d = json.loads(line)
        rf = d["roofline"]
        res[l].append((d["value"], rf["avg_launch_us"], d.get("lookup_roofline", {}).get("avg_launch_us")))
        print(l, res[l][-1], flush=True)
print(json.dumps(res))
