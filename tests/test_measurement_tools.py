"""CPU tests of the measurement plumbing the bench line depends on: the rocprofv3 trace
summary that chooses the roofline kernel (tools/rocprof_summary.py), the kernel roofline arithmetic and
the hash-matched record lookup (bench.py), and the launcher's WORLD_SIZE check."""
import json
import os
import subprocess
import sys
from pathlib import Path

import pytest

REPO = Path(__file__).resolve().parents[1]
sys.path.insert(0, str(REPO))
sys.path.insert(0, str(REPO / "tools"))

import bench  # noqa: E402
import rocprof_summary as rs  # noqa: E402

# one synthetic matvec step: the key switch of the baby steps, the Hadamard, the giant steps, the rescale
# (names as rocprofv3 prints them, durations in microseconds)
STEP = [("void fhs::k_ks_intt_h<14>(fhs::DevTables, ...)", 10), ("fhs::k_centered_x(fhs::DevTables, ...)", 2),
        ("void fhs::k_modup_h<14, 3, true>(fhs::DevTables, ...)", 50), ("fhs::k_ks_ip(fhs::DevTables, ...)", 600),
        ("fhs::k_special_x(fhs::DevTables, ...)", 5), ("void fhs::k_moddown_h<14, true, true>(...)", 400),
        ("void fhs::k_bsgs_inner<2, 16, 16>(fhs::DevTables, ...)", 1900),
        ("void fhs::k_ks_intt_h<14>(fhs::DevTables, ...)", 180), ("fhs::k_centered_x(fhs::DevTables, ...)", 60),
        ("void fhs::k_modup_h<14, 3, true>(fhs::DevTables, ...)", 1800), ("fhs::k_ks_ip(fhs::DevTables, ...)", 80),
        ("fhs::k_ks_ip_sum(fhs::DevTables, ...)", 870), ("fhs::k_giant_sum(fhs::DevTables, ...)", 97),
        ("void fhs::k_giant_final<14, false>(...)", 33), ("void fhs::k_rescale_intt<14, false>(...)", 28)]


def trace(steps, warm_scale=3.0, gap_us=1):
    """rows (start_ns, end_ns, name) of `steps` steps; the first step's kernels run warm_scale x slower"""
    rows, t = [], 0
    for s in range(steps):
        for name, us in STEP:
            d = int(us * 1000 * (warm_scale if s == 0 else 1.0))
            rows.append((t, t + d, name))
            t += d + gap_us * 1000
    return rows


def test_rocprof_summary_steady_state_and_longest_priced_kernel():
    res = rs.summarise(trace(6), 4)
    k = res["kernels"]
    assert res["steps_timed"] == 4
    # families: both ModUps (baby 50 + giant 1800 us), both key products + the giant sum (600 + 80 + 870)
    assert k["k_modup"]["ms_per_step"] == pytest.approx(1.85) and k["k_modup"]["launches_per_step"] == 2
    assert k["k_ks_ip"]["ms_per_step"] == pytest.approx(1.55)
    assert k["k_moddown"]["ms_per_step"] == pytest.approx(0.405)
    assert k["k_ks_intt"]["ms_per_step"] == pytest.approx(0.252)
    assert k["k_bsgs_inner"]["ms_per_step"] == pytest.approx(1.9)
    # the cold first step is outside the timed steps but inside the all-dispatch average
    assert k["k_bsgs_inner"]["all_dispatch_ms_per_launch"] > k["k_bsgs_inner"]["ms_per_launch"]
    assert res["longest_matvec_kernel"] == "k_bsgs_inner"   # priced kernels only: 1.9 > 1.85 > 1.55
    busy = sum(us for _, us in STEP) / 1000
    assert res["step_kernel_busy_ms_median"] == pytest.approx(busy)
    assert res["step_span_ms_median"] == pytest.approx(busy + (len(STEP) - 1) / 1000)
    with pytest.raises(SystemExit):   # fewer Hadamard dispatches than timed steps
        rs.summarise(trace(3), 4)


def test_kernel_roofline_arithmetic():
    cfg = bench.CONFIGS["cfg2"]
    l = cfg["L0"] - 1
    ab = bench.algorithmic_bytes_per_matvec("k_bsgs_inner", cfg, l)
    steps = 20
    ktimes = {"k_bsgs_inner": (steps * 1.9, steps)}   # 1.9 ms per step, one launch each
    traffic = ({"k_bsgs_inner": {"traffic_bytes_per_step": 1.02 * ab}}, "profiles/rX/pmc_traffic_cfg2.json")
    valu = ({"k_bsgs_inner": {"valu_busy": 0.34}}, "profiles/rX/pmc_valu_cfg2.json")
    rrec = {"kernels": {"k_bsgs_inner": {"ms_per_step": 2.0}}}
    r = bench.kernel_roofline("k_bsgs_inner", ktimes, steps, cfg, l, traffic, valu, rrec)
    assert r["achieved"] == pytest.approx(ab / 1.9e-3 / 1e9, rel=1e-4)
    assert r["frac"] == pytest.approx(ab / 1.9e-3 / 1e9 / bench.HBM_PEAK_GBS, rel=1e-3)
    assert r["traffic_over_algorithmic"] == pytest.approx(1.02)
    assert r["traffic"] == int(1.02 * ab) and r["valu_busy"] == 0.34
    assert r["rocprof_frac"] == pytest.approx(ab / 2.0e-3 / 1e9 / bench.HBM_PEAK_GBS, rel=1e-3)
    # ModUp: two launches per step -> bytes and traffic per launch are half the step's
    mu = bench.algorithmic_bytes_per_matvec("k_modup", cfg, l)
    r = bench.kernel_roofline("k_modup", {"k_modup": (steps * 1.8, 2 * steps)}, steps, cfg, l,
                              ({"k_modup_h": {"traffic_bytes_per_step": 1.4 * mu}}, "x"), ({}, None), None)
    assert r["launches_per_step"] == 2 and r["bytes_per_launch"] == mu // 2
    assert r["traffic"] == int(1.4 * mu / 2) and r["valu_busy"] is None and "rocprof_frac" not in r
    assert bench.kernel_roofline("k_giant_sum", {"k_giant_sum": (1.0, 20)}, steps, cfg, l, ({}, None), ({}, None),
                                 None) is None   # unpriced


def test_latest_record_needs_matching_kernel_hash(tmp_path, monkeypatch):
    for rnd, h in (("r07", "aaaa"), ("r08", "bbbb"), ("r09", "cccc")):
        d = tmp_path / "profiles" / rnd
        d.mkdir(parents=True)
        (d / "rocprof_summary_cfgT.json").write_text(json.dumps({"kernel_source_sha256_16": h, "round": rnd}))
    monkeypatch.setattr(bench, "REPO", tmp_path)
    monkeypatch.setattr(bench, "kernel_source_hash", lambda: "bbbb")
    rec, src = bench.latest_record("rocprof_summary", "cfgT")
    assert rec["round"] == "r08" and src == "profiles/r08/rocprof_summary_cfgT.json"
    monkeypatch.setattr(bench, "kernel_source_hash", lambda: "dddd")
    assert bench.latest_record("rocprof_summary", "cfgT") == (None, None)


def test_kernel_source_hash_covers_the_kernel_sources():
    """The committed records' hash is over fhs_kernels.hip and the device headers it includes."""
    h = bench.kernel_source_hash()
    assert len(h) == 16 and all(c in "0123456789abcdef" for c in h)
    src = (REPO / "fhe-spear_amd" / "csrc" / "fhs_kernels.hip").read_text()
    for inc in ("fhs_ntt.h", "fhs_buffer.h"):
        assert f'#include "{inc}"' in src


def test_bench_rejects_a_world_size_other_than_gpus():
    """--gpus N under a launcher that set WORLD_SIZE != N exits 2 before any GPU call."""
    env = dict(os.environ, WORLD_SIZE="3", RANK="0", LOCAL_RANK="0")
    r = subprocess.run([sys.executable, str(REPO / "bench.py"), "--gpus", "2"], env=env, capture_output=True,
                       text=True, timeout=120)
    assert r.returncode == 2
    assert "WORLD_SIZE=3" in r.stderr


def test_gpu_scripts_parse():
    """The GPU-box scripts (tools/gpu.sh and the rehearsal scripts) are at least valid bash."""
    for f in sorted((REPO / "tools").glob("*.sh")) + sorted((REPO / "tools" / "debug").glob("*.sh")):
        r = subprocess.run(["bash", "-n", str(f)], capture_output=True, text=True)
        assert r.returncode == 0, (f.name, r.stderr)


def test_pmc_stall_shares(tmp_path):
    """tools/pmc_stall.py: per-kernel sums over two PMC passes, per step, shares of
    SQ_WAVE_CYCLES, VALU busy against the SIMD cycles (GRBM_GUI_ACTIVE averaged over the passes carrying it)."""
    hdr = "Dispatch_Id,Kernel_Name,Counter_Name,Counter_Value\n"
    k = '"void fhs::k_modup_h<14, 3, true>(fhs::DevTables, ...)"'   # quoted, as rocprofv3 writes it
    p1 = tmp_path / "p1.csv"
    p1.write_text(hdr + "".join(f"{d},{k},{n},{v}\n" for d in (1, 2) for n, v in (
        ("SQ_WAVE_CYCLES", 1000), ("SQ_WAIT_ANY", 350), ("SQ_WAIT_INST_ANY", 350), ("SQ_ACTIVE_INST_ANY", 300),
        ("SQ_ACTIVE_INST_VALU", 2048 * 8), ("GRBM_GUI_ACTIVE", 8 * 64))))
    p2 = tmp_path / "p2.csv"
    p2.write_text(hdr + "".join(f"{d},{k},{n},{v}\n" for d in (5, 6) for n, v in (
        ("SQ_INSTS_VALU", 100), ("SQ_INSTS_LDS", 10), ("SQ_LDS_BANK_CONFLICT", 17), ("GRBM_GUI_ACTIVE", 8 * 64))))
    out = tmp_path / "stall.json"
    subprocess.run([sys.executable, str(REPO / "tools" / "pmc_stall.py"), str(out), "2", str(p1), str(p2)], check=True,
                   capture_output=True)
    rec = json.loads(out.read_text())["kernels"]["k_modup_h"]
    assert rec["launches_per_step"] == 1.0
    assert rec["share_wait_any"] == 0.35 and rec["share_active_inst_any"] == 0.3
    # per step: 2048 x 8 VALU quad-cycles x 4 over 1024 SIMDs x (512 per pass, 2 passes -> 512) / 8 cycles
    assert rec["valu_busy"] == round(2048 * 8 * 4 / (1024 * 512 / 8), 3)
    assert rec["bank_conflict_cycles_per_lds_inst"] == 1.7 and rec["lds_per_valu"] == 0.1


@pytest.mark.parametrize("record", ["r05/rehearse_n4_gloo_one_gpu.json", "r05/rehearse_n8_gloo_one_gpu_matvec_cfg5.json",
                                    "r05/rehearse_n8_gloo_one_gpu_matvec_block.json",
                                    "r05/rehearse_n2_gloo_one_gpu.json", "r06/rehearse_n2_gloo_one_gpu.json",
                                    "r06/rehearse_n4_gloo_one_gpu.json",
                                    "r06/rehearse_n8_gloo_one_gpu_full_line.json"])
def test_multi_rank_line_schema_on_the_rehearsal_records(record):
    """the fields the driver's first 8-GPU run must carry -- world size, a device record
    with its PCI bus id per rank, per-kind exchange {calls, MB, ms} for the matvec, block and cfg5 legs, the
    block in both baby-step modes, the cfg5 digest against the one-rank digest -- pinned by bench.py's own
    checker (which also stamps `schema_errors` into every line) on the committed world-2 / world-8
    rehearsals (8 gloo ranks sharing one GPU: the matvec + cfg5 legs and the matvec + block legs ran as two
    records, the ranks' memory together exceeding one GPU's 288 GB with all legs at once)."""
    res = json.loads((REPO / "profiles" / record).read_text())
    assert bench.line_schema_errors(res) == []
    if "cfg5" in record or record.startswith(("r06/rehearse_n2", "r06/rehearse_n4")):
        assert res["cfg5_chain"]["parity"]["matches_one_rank"] is True
    if record.startswith("r06/"):
        # round 6: the whole default line in one run; at world 8 with 8 ranks on one GPU the cfg5 leg runs out of
        # memory on a rank, every rank leaves it (FailureFence), the process group is re-created and the line printed
        assert res["summary"]["schema_errors"] == [] and res["parity"]["gathered_outputs"]["all_match"]
        if "n8" in record:
            f = res["leg_faults"]["cfg5"]
            assert "out of memory" in f["error"] and len(f["failed_ranks"]) >= 1
            assert sorted(f["failed_ranks"] + f["abandoned_ranks"]) == list(range(8)) and not f["unresponsive_ranks"]
            assert res["cfg5_chain"]["error"] == f["error"]
    if res.get("rwkv_block"):
        assert res["rwkv_block"]["baby_broadcast"]["baby_mode"] == "broadcast"


def test_multi_rank_line_schema_reports_what_is_missing():
    res = json.loads((REPO / "profiles" / "r05" / "rehearse_n8_gloo_one_gpu_matvec_block.json").read_text())
    res["ranks"]["devices"] = res["ranks"]["devices"][:7]
    del res["rwkv_block"]["baby_broadcast"]
    res["exchange_per_step"]["gather"].pop("ms")
    err = bench.line_schema_errors(res)
    assert len(err) == 3 and any("pci_bus_id" in e for e in err) and any("baby_broadcast" in e for e in err)
