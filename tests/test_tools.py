"""CPU checks of the measurement tools' pure logic (the GPU sessions themselves run under tools/gpu.sh)."""
import importlib.util
import os

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def _tool(name):
    spec = importlib.util.spec_from_file_location(name, os.path.join(ROOT, "tools", f"{name}.py"))
    mod = importlib.util.module_from_spec(spec)
    spec.loader.exec_module(mod)
    return mod


def test_tune_gemms_merge_replaces_retuned_rows_in_place_and_appends_new_ones():
    tg = _tool("tune_gemms")
    committed = [
        "Validator,PT_VERSION,2.10.0\n",
        "Validator,GCN_ARCH_NAME,gfx950:sramecc+:xnack-\n",
        "GemmTunableOp_BFloat16_TN,tn_6144_8192_4096_ld_4096_4096_6144,Gemm_Hipblaslt_618611,0.268148\n",
        "GemmTunableOp_BFloat16_TN,tn_128256_8192_4096_ld_4096_4096_128256,Gemm_Hipblaslt_618611,5.68609",
    ]
    results = [
        ("GemmTunableOp_BFloat16_TN", "tn_6144_8192_4096_ld_4096_4096_6144", "Gemm_Rocblas_618614", 0.27),
        ("GemmTunableOp_BFloat16_NN", "nn_4096_8192_6144_ld_4096_6144_4096", "Default", 0.3),
    ]
    rows = tg.merge_results(committed, results)
    assert rows[:2] == committed[:2]  # validators untouched, first
    assert rows[2] == "GemmTunableOp_BFloat16_TN,tn_6144_8192_4096_ld_4096_4096_6144,Gemm_Rocblas_618614,0.27\n"
    assert rows[3] == committed[3] + "\n"  # skipped shape (LM head) keeps its committed winner
    assert rows[4] == "GemmTunableOp_BFloat16_NN,nn_4096_8192_6144_ld_4096_6144_4096,Default,0.3\n"
    assert len(rows) == 5 and all(r.endswith("\n") for r in rows)


def test_stream_gaps_sums_same_stream_gaps_per_kernel_pair_inside_the_step_window():
    sg = _tool("stream_gaps")
    ns = 1000  # timestamps in ns
    rows = [
        (0, 1 * ns, "kop::clip_coef_kernel", "0"),            # step 1 starts
        (2 * ns, 50 * ns, "gemm_a", "0"),
        (62 * ns, 70 * ns, "gelu_bwd", "0"),                  # 12 us after gemm_a on its stream
        (51 * ns, 90 * ns, "wgrad", "1"),                     # other stream: not a gap of stream 0
        (101 * ns, 102 * ns, "kop::clip_coef_kernel", "0"),   # step 2 starts
        (104 * ns, 150 * ns, "gemm_a", "0"),
        (161 * ns, 170 * ns, "gelu_bwd", "0"),                # 11 us
        (172 * ns, 173 * ns, "tiny", "0"),                    # 2 us: below --min-us
        (200 * ns, 201 * ns, "kop::clip_coef_kernel", "0"),   # end of the window
    ]
    res = sg.stream_gaps(rows, steps=2, min_us=5.0)
    s0 = res["0"]
    assert abs(s0["pairs"][("gemm_a", "gelu_bwd")] - 11.5) < 1e-9  # us per step
    assert s0["counts"][("gemm_a", "gelu_bwd")] == 2
    # plus gelu_bwd -> the second step's clip_coef (31 us, once); the window ends at the last clip_coef
    assert set(s0["pairs"]) == {("gemm_a", "gelu_bwd"), ("gelu_bwd", "kop::clip_coef_kernel")}
    assert abs(s0["gap_ms"] - (12 + 11 + 31) / 2 / 1e3) < 1e-12
    assert res["1"]["gap_ms"] == 0.0


def test_gpu_telemetry_parses_sysfs_and_summarizes(tmp_path):
    from kubeoperator_amd.train import gpu_telemetry as gt

    assert gt.parse_sclk("0: 500Mhz\n1: 1650Mhz\n2: 2400Mhz *\n") == 2400
    assert gt.parse_sclk("0: 500Mhz\n1: 1918Mhz *\n2: 2400Mhz\n") == 1918
    assert gt.parse_sclk("0: 500Mhz\n") is None
    dev, hw = tmp_path / "dev", tmp_path / "dev" / "hwmon" / "hwmon3"
    hw.mkdir(parents=True)
    (dev / "pp_dpm_sclk").write_text("0: 500Mhz\n1: 1900Mhz *\n")
    (hw / "power1_average").write_text("1312000000\n")
    s = gt.PowerClockSampler(where=(str(dev), str(hw)))
    t, p, c = s.read()
    assert (p, c) == (1312.0, 1900)
    s.samples = [(0, 1300.0, 1900), (1, 1320.0, None), (2, None, 1920)]
    s.where = (str(dev), str(hw))
    r = s.stop()
    assert r["power_w"] == {"n": 2, "mean": 1310.0, "min": 1300.0, "max": 1320.0}
    assert r["sclk_mhz"]["n"] == 2 and r["sclk_mhz"]["max"] == 1920
    assert gt.PowerClockSampler(where=()).start().stop() is None  # no sysfs: no thread, no record
