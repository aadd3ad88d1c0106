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
