"""Where does the short-window deficit of the driver's 20/5 bench come from? bench.py runs of
(steps, warmup) = (20, 5), (20, 20), (40, 5), (100, 10), (20, 5 + 100 untimed), interleaved over
rounds in separate processes (as the driver runs it), one JSON line per run.

Usage (GPU box): python scripts/bench_windows.py [--rounds 2]
"""
import argparse
import json
import os
import subprocess
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
CONFIGS = [(20, 5), (20, 20), (40, 5), (100, 10), (20, 105)]


def main():
    p = argparse.ArgumentParser()
    p.add_argument("--rounds", type=int, default=2)
    a = p.parse_args()
    for r in range(a.rounds):
        for steps, warm in CONFIGS:
            out = subprocess.run([sys.executable, "bench.py", "--steps", str(steps), "--warmup", str(warm)], cwd=ROOT,
                                 capture_output=True, text=True, timeout=300)
            if out.returncode != 0:
                print(out.stderr[-2000:], file=sys.stderr)
                return out.returncode
            d = json.loads(out.stdout.strip().splitlines()[-1])
            print(json.dumps({"round": r, "steps": steps, "warmup": warm, "img_s": d["value"],
                              "ms_per_step": d["ms_per_step"],
                              "sclk_mhz": (d.get("calibration") or {}).get("sclk_mhz")}), flush=True)
    return 0


if __name__ == "__main__":
    sys.exit(main())
