"""CPU tests of the C-ABI library: it loads, exports every symbol include/lamm_hip.h
declares, its traits match the format contract, and argument validation behaves --
no compute calls (there is no GPU here)."""
import ctypes
import os
import re

import numpy as np
import pytest

import lamm_amd as la
import oracle_lib as ol

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
HEADER = os.path.join(ROOT, "include", "lamm_hip.h")
NO_GPU = la.device_count() == 0


def declared_symbols():
    text = open(HEADER).read()
    text = re.sub(r"/\*.*?\*/", "", text, flags=re.S)
    return sorted(set(re.findall(r"\b(lamm_\w+)\s*\(", text)))


def test_header_symbols_exported():
    syms = declared_symbols()
    assert {"lamm_can_mul_mat", "lamm_mul_mat", "lamm_get_opt_level", "lamm_hip_matmul"} <= set(syms)
    for s in syms:
        assert hasattr(la.lib, s), f"{s} declared in include/lamm_hip.h but not exported"


def test_struct_layouts_match_b2430():
    assert ctypes.sizeof(la.GgmlTensor) == 368
    assert la.GgmlTensor.data.offset == 280 and la.GgmlTensor.src.offset == 160
    assert la.GgmlTensor.ne.offset == 16 and la.GgmlTensor.nb.offset == 48
    assert ctypes.sizeof(la.GgmlComputeParams) == 32 and la.GgmlComputeParams.wdata.offset == 24
    assert ctypes.sizeof(la.Matrix) == 32 and la.Matrix.ld.offset == 24  # == struct Matrix


@pytest.mark.skipif(not os.path.isdir("/root/reference/llama.cpp-b2430"), reason="reference headers absent")
def test_struct_layouts_against_reference_header(tmp_path):
    src = tmp_path / "abi.c"
    src.write_text(
        '#include "ggml.h"\n#include <stdio.h>\n#include <stddef.h>\n'
        'int main(){printf("%zu %zu %zu %zu %zu %zu\\n", sizeof(struct ggml_tensor),'
        ' offsetof(struct ggml_tensor,data), offsetof(struct ggml_tensor,src), offsetof(struct ggml_tensor,nb),'
        ' sizeof(struct ggml_compute_params), offsetof(struct ggml_compute_params,wdata));}\n')
    exe = tmp_path / "abi"
    import subprocess
    subprocess.run(["gcc", "-I/root/reference/llama.cpp-b2430", str(src), "-o", str(exe)], check=True)
    out = subprocess.run([str(exe)], check=True, capture_output=True, text=True).stdout.split()
    assert list(map(int, out)) == [368, 280, 160, 48, 32, 24]


def test_traits_match_oracle():
    o = ol.Oracle()
    for t in [ol.F32, ol.Q4_0, ol.Q4_1, ol.Q5_0, ol.Q5_1, ol.Q8_0, ol.Q8_1, ol.Q2_K, ol.Q8_K] + ol.KQ_TYPES + [ol.F16]:
        assert la.blck_size(t) == o.block_elems(t)
        assert la.type_size(t) == o.block_bytes(t)
    for t in ol.A_TYPES + ol.KQ_TYPES:
        assert la.vec_dot_type(t) == o.vec_dot_type(t)
    # F16 and the k-quants are SURVEY §8f additions beyond the reference's lamm pairs
    # (src/loongarch_matmul.cpp:37-52); Q3_K (11) stays unsupported
    assert la.vec_dot_type(1) == 1 and la.vec_dot_type(11) == -1


def _mats(wtype=la.Q4_0, M=16, N=1, kb=128, lda=None):
    vt = la.vec_dot_type(wtype)
    A = la.Matrix(0x100000, wtype, M, kb, lda if lda is not None else kb)
    B = la.Matrix(0x200000, vt, kb, N, kb)
    C = la.Matrix(0x300000, la.F32, M, N, M)
    return A, B, C


def _rc(A, B, C):
    return la.lib.lamm_hip_matmul(ctypes.byref(A), ctypes.byref(B), ctypes.byref(C), None)


def test_validation_errors():
    A, B, C = _mats()
    B.type = la.Q8_1
    assert _rc(A, B, C) == la.LAMM_ERR_TYPE
    A, B, C = _mats()
    A.type = la.F16            # F16 weights are supported, but only against F16 activations
    assert _rc(A, B, C) == la.LAMM_ERR_TYPE      # B is still q8_0: not vec_dot_type(F16)
    B.type = la.F16
    assert _rc(A, B, C) in (la.LAMM_OK, la.LAMM_ERR_NODEV, la.LAMM_ERR_SHAPE)
    A, B, C = _mats()
    A.type = 11                # Q3_K: no kernel
    assert _rc(A, B, C) == la.LAMM_ERR_TYPE
    A, B, C = _mats()
    B.row = 64
    assert _rc(A, B, C) == la.LAMM_ERR_SHAPE
    A, B, C = _mats(kb=3)          # q4_0 row of 3 blocks = 54 bytes: not a 16-byte pitch
    assert _rc(A, B, C) == la.LAMM_ERR_ALIGN
    A, B, C = _mats(kb=3, lda=8)   # pitched to 144 bytes: accepted
    assert _rc(A, B, C) in (la.LAMM_OK, la.LAMM_ERR_NODEV)


def test_group_validation_errors():
    """lamm_hip_matmul_group: 1..LAMM_GROUP_MAX weights; a group the one-launch form cannot take (two
    columns, mixed types) goes through the per-weight calls and their own validation."""
    A, B, C = _mats()
    rc = la.lib.lamm_hip_matmul_group((la.Matrix * 5)(*([A] * 5)), 5, ctypes.byref(B), (la.Matrix * 5)(*([C] * 5)),
                                      la.ORDER_REFERENCE, None)
    assert rc == la.LAMM_ERR_SHAPE
    rc = la.lib.lamm_hip_matmul_group((la.Matrix * 1)(A), 0, ctypes.byref(B), (la.Matrix * 1)(C), 0, None)
    assert rc == la.LAMM_ERR_SHAPE
    if not NO_GPU:   # the calls below reach the per-weight path with placeholder pointers
        return
    A2, B2, C2 = _mats()
    B2.row = 64                       # a shape error in the second weight's call
    rc = la.lib.lamm_hip_matmul_group((la.Matrix * 2)(A, A2), 2, ctypes.byref(B2), (la.Matrix * 2)(C, C2), 0, None)
    assert rc in (la.LAMM_ERR_SHAPE, la.LAMM_ERR_NODEV)
    A3, _, _ = _mats()
    A3.type = 11                      # Q3_K: no kernel, even inside a group
    rc = la.lib.lamm_hip_matmul_group((la.Matrix * 2)(A, A3), 2, ctypes.byref(B), (la.Matrix * 2)(C, C), 0, None)
    assert rc in (la.LAMM_ERR_TYPE, la.LAMM_ERR_NODEV)


@pytest.mark.skipif(not NO_GPU, reason="checks the no-GPU behaviour")
def test_no_gpu_behaviour():
    A, B, C = _mats()
    assert _rc(A, B, C) == la.LAMM_ERR_NODEV
    assert la.get_opt_level() == 0
    import ggml_emu
    src0 = ggml_emu.Tensor(la.Q4_0, [64, 4], data=np.zeros(4 * 36, np.uint8))
    src1 = ggml_emu.Tensor(la.F32, [64, 2], data=np.zeros(128, np.float32))
    dst = ggml_emu.mul_mat_node(src0, src1)
    # no GPU: the hook declines and ggml keeps its CPU loop
    assert ggml_emu.compute(dst, nth=2) is False


def test_build_id_matches_tree():
    """Provenance: the loaded liblamm_hip.so was built from exactly this tree's sources
    (Makefile BUILD_ID vs lamm_amd.source_build_id()); a stale prebuilt library fails here."""
    assert la.build_id() == la.source_build_id(), (
        f"liblamm_hip.so build id {la.build_id()} != sources {la.source_build_id()}: rebuild with make -C la-llama.cpp_amd")


@pytest.mark.parametrize("align", [1, 4, 16, 128, 256])
def test_shard_rows_cover_every_row_once(align):
    """lamm_hip_shard_rows (the multi-GPU row split): contiguous slabs in rank order
    covering [0, M) exactly once, boundaries on `align`-row tiles, slab sizes differing by at most
    one tile -- unlike the reference's M / nth split (src/lamm_impl.hpp:38-43), which drops the
    M % nth tail rows (SURVEY §8a defect 1)."""
    for M in [0, 1, 5, 63, 64, 65, 4095, 4096, 4097, 11008, 32000]:
        for world in [1, 2, 3, 4, 7, 8]:
            slabs = [la.shard_rows(M, world, r, align) for r in range(world)]
            pos = 0
            for r0, rows in slabs:
                assert r0 == pos and rows >= 0
                pos += rows
                if rows and r0 + rows < M:
                    assert (r0 + rows) % align == 0
            assert pos == M
            tiles = [-(-rows // align) for _, rows in slabs]
            assert max(tiles) - min(tiles) <= 1


def test_env_switches_read_once_and_reloaded(monkeypatch):
    """The library reads its LAMM_* switches once (lamm_knobs.cpp) and again only on
    lamm_hip_reload_env / lamm_hip_boundary_reset; the Python binding re-syncs when os.environ's
    LAMM_* part changes.  LAMM_OPT_LEVEL=0 is visible through lamm_get_opt_level() (0 without a
    GPU either way, so this checks the sync path, and on a GPU box the switch itself)."""
    base = la.get_opt_level()
    monkeypatch.setenv("LAMM_OPT_LEVEL", "0")
    assert la.get_opt_level() == 0          # _sync_env saw the change and reloaded
    monkeypatch.delenv("LAMM_OPT_LEVEL")
    assert la.get_opt_level() == base
    # a raw change without the binding's sync stays invisible until reload_env()
    os.environ["LAMM_OPT_LEVEL"] = "0"
    try:
        assert la.lib.lamm_get_opt_level() == base
        la.reload_env()
        assert la.lib.lamm_get_opt_level() == 0
    finally:
        del os.environ["LAMM_OPT_LEVEL"]
        la.reload_env()
    assert la.lib.lamm_get_opt_level() == base


def test_no_getenv_on_launch_paths():
    """Product-path hygiene: only lamm_knobs.cpp reads the environment; ablation switches
    (LAMM_GEMM_VARIANT, LAMM_GEMM_SKIP_PREP, ...) exist only in the LAMM_AB_VARIANTS build."""
    csrc = os.path.join(ROOT, "la-llama.cpp_amd", "csrc")
    for f in sorted(os.listdir(csrc)):
        if not f.endswith((".hip", ".cpp", ".h")) or f == "lamm_knobs.cpp":
            continue
        depth = 0
        for ln in open(os.path.join(csrc, f)):
            if ln.startswith("#ifdef LAMM_AB_VARIANTS"):
                depth += 1
            elif depth and ln.startswith("#endif"):
                depth -= 1
            elif "getenv(" in ln:
                assert depth > 0, f"{f}: getenv outside the variant build: {ln.strip()}"


def test_engine_choice(monkeypatch):
    """lamm_hip_engine reports the dispatch lamm_hip_matmul* makes (host logic, no device): the
    decode GEMV up to each type's widest N, then the prefill engines; LAMM_GEMV_MAX_N overrides
    the per-type width, with 0 and 1 both meaning N = 1 only ('0' had silently
    become 'unset' in the library while the binding read it as 1)."""
    for k in ("LAMM_GEMV_MAX_N", "LAMM_GEMM_PATH", "LAMM_FP6_SPLIT", "LAMM_FP6_SUB", "LAMM_DENSE_GEMM", "LAMM_KQ_GEMM"):
        monkeypatch.delenv(k, raising=False)
    e = la.gemm_engine
    assert e("q4_0", 4096, 1, 4096) == "gemv" and e("q4_0", 4096, 8, 4096) == "gemv"
    assert e("q2_k", 4096, 5, 4096) == "gemv" and e("q2_k", 4096, 6, 4096) == "superblock"
    assert e("q6_k", 4096, 4, 4096) == "gemv" and e("q6_k", 4096, 5, 4096) == "superblock"
    assert e("f16", 4096, 5, 4096) == "dense" and e("f32", 512, 512, 512) == "dense"
    # BASELINE config 3: the fp6 engine's 128x64 K-group tiles fill the chip with stationary weights;
    # q5_1 / q8_0 prefill on the dequantizing f16 engine once its tiles fill half the chip, the
    # exact MFMA-i8 engine (split-K) below that
    assert e("q4_0", 4096, 512, 4096, stationary=True) == "fp6"
    assert e("q5_1", 4096, 512, 4096, stationary=True) == "fp6" and e("q5_1", 4096, 512, 4096) == "dq16"
    assert e("q8_0", 4096, 512, 4096) == "dq16" and e("q8_0", 4096, 64, 4096) == "i8"
    assert e("q4_0", 4096, 9, 4096) in ("fp6", "i8")
    assert e("q5_0", 4096, 512, 4096, b_f32=True) == e("q5_0", 4096, 512, 4096)
    assert e("q4_0", 4096, 8, 4096, b_f32=True) == "gemv"
    assert e(11, 4096, 1, 4096) == "" and e("q4_0", 4096, 1, 100) == ""
    monkeypatch.setenv("LAMM_GEMV_MAX_N", "0")
    assert e("q4_0", 4096, 1, 4096) == "gemv" and e("q4_0", 4096, 2, 4096) != "gemv"
    monkeypatch.setenv("LAMM_GEMV_MAX_N", "1")
    assert e("q4_0", 4096, 2, 4096) != "gemv"
    # F32 activations stay on the fused GEMV up to 8 columns whatever the override
    assert e("q4_0", 4096, 8, 4096, b_f32=True) == "gemv"
    monkeypatch.setenv("LAMM_GEMV_MAX_N", "4")
    assert e("q4_0", 4096, 4, 4096) == "gemv" and e("q4_0", 4096, 5, 4096) != "gemv"
    monkeypatch.delenv("LAMM_GEMV_MAX_N")
    monkeypatch.setenv("LAMM_GEMM_PATH", "i8")
    assert e("q4_0", 4096, 512, 4096, stationary=True) == "i8"
    monkeypatch.setenv("LAMM_GEMM_PATH", "fp6")
    assert e("q4_0", 4096, 64, 4096) == "fp6"
