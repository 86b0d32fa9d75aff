"""The trace tools behind the round-6 timing claims (scripts/step_timeline.py, scripts/ramp_table.py)
on a synthetic rocpd database: step splitting at the step-head kernel, per-queue busy / idle time,
the --last table, and the early-vs-late per-kernel attribution. CPU only."""
import os
import sqlite3
import subprocess
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def _db(path, steps):
    """steps: list of (main kernels [(name, dur_us, gap_before_us)], side kernels [(name, start_off, dur)])."""
    c = sqlite3.connect(path)
    c.execute("create table rocpd_info_kernel_symbol (id integer, display_name text)")
    c.execute("create table rocpd_kernel_dispatch (id integer, kernel_id integer, start integer, end integer, "
              "queue_id integer)")
    names = {}
    did = 0
    t = 1_000_000
    for main, side in steps:
        t0 = t
        for name, dur, gap in main:
            t += int(gap * 1e3)
            kid = names.setdefault(name, len(names) + 1)
            c.execute("insert into rocpd_kernel_dispatch values (?,?,?,?,?)", (did, kid, t, t + int(dur * 1e3), 3))
            did += 1
            t += int(dur * 1e3)
        for name, off, dur in side:
            kid = names.setdefault(name, len(names) + 1)
            s0 = t0 + int(off * 1e3)
            c.execute("insert into rocpd_kernel_dispatch values (?,?,?,?,?)", (did, kid, s0, s0 + int(dur * 1e3), 1))
            did += 1
    # a final head so the last step closes
    kid = names.setdefault("conv0_fwd_kernel<true>(float const*)", len(names) + 1)
    c.execute("insert into rocpd_kernel_dispatch values (?,?,?,?,?)", (did, kid, t, t + 1000, 3))
    for n, i in names.items():
        c.execute("insert into rocpd_info_kernel_symbol values (?,?)", (i, n))
    c.commit()
    c.close()


def _step(gemm_us, gap_us=0.0):
    main = [("conv0_fwd_kernel<true>(float const*)", 10.0, 0.0), ("bn_apply_kernel(float const*)", 5.0, gap_us),
            ("(anonymous namespace)::conv_gemm_kernel<64, 64, 0, 64, 6, false, 0, 4>(CsConvArgs)", gemm_us, 0.0)]
    side = [("conv_gemm_kernel<64, 64, 2, 16, 6, false, 0, 1>(CsConvArgs)", 2.0, 12.0)]
    return main, side


def _run(script, *args):
    r = subprocess.run([sys.executable, os.path.join(ROOT, "scripts", script), *args], capture_output=True, text=True,
                       timeout=60)
    assert r.returncode == 0, r.stderr
    return r.stdout


def test_step_timeline_busy_idle_and_last_table(tmp_path):
    d = tmp_path / "trace"
    d.mkdir()
    _db(str(d / "run_results.db"), [_step(20.0, gap_us=3.0), _step(20.0), _step(30.0, gap_us=7.0)])
    out = _run("step_timeline.py", str(d), "--last", "3")
    lines = out.splitlines()
    assert lines[0].startswith("# last 3 steps")
    rows = [tuple(float(x) for x in l.split()) for l in lines[1:4]]
    # span / busy / idle per step: head 10 + gap + apply 5 + gemm
    assert rows[0] == (38.0, 35.0, 3.0) and rows[1] == (35.0, 35.0, 0.0) and rows[2] == (52.0, 45.0, 7.0)
    # the detail is the step with the least main-queue idle, with both queues
    assert "# one step: 4 dispatches, span 35.0 us" in out
    assert "# queue 3: idle between its dispatches 0.0 us" in out
    assert "main-queue busy by class (us): conv_gemm 20.0" in out


def test_ramp_table_attributes_the_span_delta_to_kernels(tmp_path):
    d = tmp_path / "ramp"
    d.mkdir()
    # 12 steps: the GEMM takes 30 us in steps 0-5 and 20 us after
    _db(str(d / "run_results.db"), [_step(30.0 if i < 6 else 20.0) for i in range(12)])
    out = _run("ramp_table.py", str(d), "--early", "1:4", "--late", "7:10")
    assert "delta +10.0 us" in out
    gemm = next(l for l in out.splitlines() if l.startswith("conv_gemm_kernel<64, 64, 0, 64"))
    f = gemm.split()
    assert f[-6] == "main" and float(f[-5]) == 30.0 and float(f[-4]) == 20.0 and float(f[-3]) == 10.0
