"""The profile readers behind docs/PERF_NOTES.md (scripts/busy_clock.py, scripts/step_timeline.py,
scripts/pmc_summary.py) on synthetic rocprofv3 CSVs of the layout rocprofv3 writes."""
import csv
import importlib.util
import os

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def _load(name):
    spec = importlib.util.spec_from_file_location(name, os.path.join(ROOT, "scripts", f"{name}.py"))
    mod = importlib.util.module_from_spec(spec)
    spec.loader.exec_module(mod)
    return mod


def _write(path, header, rows):
    with open(path, "w", newline="") as f:
        w = csv.writer(f)
        w.writerow(header)
        w.writerows(rows)


def _trace(tmp_path, kernels):
    """kernels: [(dispatch id, name, start ns, end ns)] -> run_kernel_trace.csv"""
    _write(tmp_path / "run_kernel_trace.csv",
           ["Dispatch_Id", "Kernel_Name", "Start_Timestamp", "End_Timestamp"],
           [[d, n, s, e] for d, n, s, e in kernels])


def test_busy_clock_per_dispatch(tmp_path, capsys):
    # two dispatches of 1 ms: GRBM_GUI_ACTIVE = 8 XCDs x 2.0e6 cycles -> 2.0 GHz; MFMA busy
    # cycles = 0.5 x 2.0e6 x 1024 SIMDs -> busy 0.5
    _trace(tmp_path, [(1, "void tdc::k<1>(int)", 0, 1_000_000),
                      (2, "void tdc::k<1>(int)", 2_000_000, 3_000_000),
                      (3, "other_kernel", 3_000_000, 3_100_000)])
    rows = []
    for d in (1, 2):
        rows += [[d, "void tdc::k<1>(int)", "GRBM_GUI_ACTIVE", 16.0e6],
                 [d, "void tdc::k<1>(int)", "SQ_VALU_MFMA_BUSY_CYCLES", 0.5 * 2.0e6 * 1024]]
    rows.append([3, "other_kernel", "GRBM_GUI_ACTIVE", 1.0e5])
    _write(tmp_path / "run_counter_collection.csv",
           ["Dispatch_Id", "Kernel_Name", "Counter_Name", "Counter_Value"], rows)
    _load("busy_clock").main(str(tmp_path), r"tdc::k", 2.0e12)
    out = capsys.readouterr().out
    assert out.count("dispatch ") == 2 and "other_kernel" not in out
    assert "busy 0.500" in out and "clock 2.000 GHz" in out and "2.000 PF/s" in out
    assert "2 dispatches" in out


def test_step_timeline_splits_steps_at_the_assign(tmp_path, capsys):
    us = 1000
    _trace(tmp_path, [(1, "void tdc::assign_ring3_kernel<1>(x)", 0, 100 * us),
                      (2, "void tdc::update_kernel(x)", 100 * us, 110 * us),
                      (3, "void tdc::assign_ring3_kernel<1>(x)", 115 * us, 215 * us),
                      (4, "void tdc::update_kernel(x)", 215 * us, 225 * us),
                      (5, "void tdc::assign_ring3_kernel<1>(x)", 230 * us, 330 * us)])
    _load("step_timeline").main(str(tmp_path), "ring3", 2)
    out = capsys.readouterr().out
    assert out.count("-- step") == 2
    assert "115.0 us start to start, kernels 110.0 us" in out  # 5 us idle before the next step
    assert "gap    0.0" in out and "update_kernel" in out


@pytest.mark.parametrize("name,short", [
    ("void tdc::bigd::assign_bigd_kernel<tdc::bigd::OpFp8, 768, 8, 3, 0, 2, false>(unsigned char const*)",
     "tdc::bigd::assign_bigd_kernel<tdc::bigd::OpFp8, 768, 8, 3, 0, 2, false>"),
    ("void tdc::segsum_kernel<float, float, 4, 32, true>(float const*)",
     "tdc::segsum_kernel<float, float, 4, 32, true>"),
    # a mangled name (rocprofv3 prints some that way) is kept whole
    ("_ZN3tdc12_GLOBAL__N_121x3_compact_kernelEPKilPiS3_",
     "_ZN3tdc12_GLOBAL__N_121x3_compact_kernelEPKilPiS3_"),
])
def test_pmc_summary_keeps_nested_kernel_names(name, short):
    # kernels in a nested namespace are told apart (round 6: 'tdc::bigd' had merged the
    # fp8 quantiser with the assign kernel)
    assert _load("pmc_summary").short(name) == short[:70]
