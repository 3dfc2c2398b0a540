"""bench.py's roofline pricing on CPU (no GPU): each kernel's algorithmic
FLOPs split by the MFMA arithmetic it runs, and frac = sum(F_i / P_i) / t
(VERDICT r4 "price the roofline on the arithmetic the kernel
runs").  The producer / consumer kernel at the north-star shape prices its
QKV projection at the int8 peak and its attention at the fp16 peak."""
import os
import sys

import pytest

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import bench  # noqa: E402
import bertlib  # noqa: E402

HP = bertlib.SHAPES["minilm"]
PC = {"qkva_ntw": 0, "i8_up": 1, "i8_o": 0, "i8_down": 1}  # the Q4_0 MiniLM defaults of rounds 4-5 (O split-fp16)


def test_qkv_attention_mixed_price():
    parts = bench.kernel_parts("qkv_attention", 1024, 128, HP, PC, "q4_0")
    assert [p for _, p in parts] == [bench.PEAK_INT8_TOPS, bench.PEAK_FP16_TFLOPS]
    f_qkv, f_att = (f for f, _ in parts)
    assert f_qkv == pytest.approx(115.964e9, rel=1e-4) and f_att == pytest.approx(25.770e9, rel=1e-4)
    t = 338e-6
    r = bench.mixed_roofline(parts, t)
    ideal = f_qkv / (bench.PEAK_INT8_TOPS * 1e12) + f_att / (bench.PEAK_FP16_TFLOPS * 1e12)
    assert r["frac"] == pytest.approx(ideal / t, abs=1e-4)
    assert r["achieved"] / r["peak"] == pytest.approx(r["frac"], rel=1e-3)
    assert r["peak_dtype"] == "int8+fp16"
    assert 0.09 < r["frac"] < 0.11  # the round-5 figure at 338 us


def test_projection_forms_follow_the_library():
    # FFN-up on int8 where the library says so, fp16 where it does not, fp32 for F32 weights
    assert bench.kernel_parts("gemm_up_gelu", 8, 128, HP, PC, "q4_0")[0][1] == bench.PEAK_INT8_TOPS
    assert bench.kernel_parts("gemm_o_ln", 8, 128, HP, PC, "q4_0")[0][1] == bench.PEAK_FP16_TFLOPS
    assert bench.kernel_parts("gemm_up_gelu", 8, 128, HP, {}, "f16")[0][1] == bench.PEAK_FP16_TFLOPS
    assert bench.kernel_parts("gemm_up_gelu", 8, 128, HP, {}, "f32")[0][1] == bench.PEAK_FP32_MFMA_TFLOPS
    assert bench.kernel_parts("gemm_qkv", 8, 128, HP, {"qkva_ntw": 2}, "q4_1")[0][1] == bench.PEAK_FP16_TFLOPS
    assert bench.kernel_parts("embed_ln", 8, 128, HP, PC, "q4_0") == []
    assert bench.dtype_label("q4_0", PC) == "int8+fp16"
    assert bench.dtype_label("f16", {}) == "fp16"
    assert "qkv/up/down on int8 MFMA" in bench.dtype_note("q4_0", PC)


def test_int8_qkv_gemm_priced_by_resolved_choice():
    """option i8=qkv puts the unfused QKV GEMM on the int8 MFMA with
    the head-pair fused kernel (qkva_ntw != 0); the library reports it as
    i8_qkv, and bench prices it at the int8 peak (qkva_ntw alone would say fp16)."""
    arith = {"qkva_ntw": 2, "i8_qkv": 1, "i8_up": 1, "i8_o": 0, "i8_down": 0}
    assert bench.kernel_parts("gemm_qkv", 8, 512, bertlib.SHAPES["bge-large"], arith, "q4_1")[0][1] == \
        bench.PEAK_INT8_TOPS
    assert "qkv/up on int8 MFMA" in bench.dtype_note("q4_1", arith)
    off = dict(arith, i8_qkv=0, i8_up=0)
    assert bench.kernel_parts("gemm_qkv", 8, 512, bertlib.SHAPES["bge-large"], off, "q4_1")[0][1] == \
        bench.PEAK_FP16_TFLOPS
    assert bench.dtype_label("q4_1", off) == "fp16"
    # the pc kernel reports i8_qkv = 1 with qkva_ntw = 0
    assert bench.kernel_parts("gemm_qkv", 8, 128, HP, dict(PC, i8_qkv=1), "q4_0")[0][1] == bench.PEAK_INT8_TOPS
