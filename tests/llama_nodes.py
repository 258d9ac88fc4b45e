"""Node-level parity inside llama.cpp-b2430's real graph.

`llama_e2e --dump-mm DIR` writes the MUL_MAT nodes of block 0, the last block and the output
projection of one prefill and one decode step, each with its operands exactly as ggml handed them to
the mul_mat (integration/llama_e2e.cpp mm_cb).  check_nodes() recomputes every node with the oracle
from those same operands -- src1 quantized to the weight's vec_dot_type the way ggml's INIT does it
(q8_0 with the AVX2 from_float rounding, q8_K, f16) -- and returns each node's error
|c - c_ref| / max(|c_ref|, sum_k |a_k b_k|), the north-star bar.

Test infrastructure: only the tests import this (it drives the oracle).
"""
import json
import os

import numpy as np

import oracle_lib as ol

ORACLE = ol.Oracle()
KIND = {"attn_q": "wq", "attn_k": "wk", "attn_v": "wv", "attn_output": "wo", "ffn_gate": "w1", "ffn_down": "w2",
        "ffn_up": "w3"}


def node_kind(src0):
    if src0 == "output.weight":
        return "output"
    if src0.startswith("k-"):
        return "KQ"
    if src0.startswith("v-"):
        return "KQV"
    part = src0.split(".")
    return KIND.get(part[2], part[2]) if len(part) > 2 else src0


def layer_of(src0):
    if src0 == "output.weight":
        return -1
    if src0[:2] in ("k-", "v-"):
        return int(src0[2:])
    return int(src0.split(".")[1])


AVX_TYPES = (ol.Q4_0, ol.Q4_1, ol.Q5_0, ol.Q5_1, ol.Q6_K, ol.F16)   # lo_mul_mat_avx: the reference's x86 order


def check_node(d, ent):
    """(worst |c - c_ref| / max(|c_ref|, sum |a b|) against the oracle's scalar order, whether c is
    bit-identical to the reference's x86 float order -- None for types without that restatement)"""
    t0, t1 = ent["type0"], ent["type1"]
    K, M, ne02, ne03 = ent["ne0"]
    _, N, ne12, ne13 = ent["ne1"]
    assert ent["ne1"][0] == K and ent["ne"][:2] == [M, N], ent
    vt = ORACLE.vec_dot_type(t0)
    arow = ORACLE.row_bytes(t0, K)
    A = np.fromfile(os.path.join(d, ent["src0_file"]), np.uint8).reshape(ne03, ne02, M * arow)
    X = np.fromfile(os.path.join(d, f"{ent['idx']}_src1.bin"), np.float32).reshape(ne13, ne12, N, K)
    C = np.fromfile(os.path.join(d, f"{ent['idx']}_dst.bin"), np.float32).reshape(ne13, ne12, N, M)
    assert t1 == ol.F32
    flavour = ol.QUANT_AVX if vt in (ol.Q8_0, ol.Q8_1) else ol.QUANT_REF
    worst = 0.0
    exact = True if t0 in AVX_TYPES else None
    for i13 in range(ne13):
        for i12 in range(ne12):
            a = A[i13 // (ne13 // ne03), i12 // (ne12 // ne02)]
            b = ORACLE.quantize(vt, X[i13, i12], flavour)
            ref = ORACLE.mul_mat(t0, M, N, K, a, b)
            Ad = ORACLE.dequantize(t0, a, M, K)
            Bd = ORACLE.dequantize(vt, b, N, K)
            absdot = (np.abs(Bd) @ np.abs(Ad).T).astype(np.float64)
            denom = np.maximum(np.maximum(np.abs(ref.astype(np.float64)), absdot), 1e-30)
            err = np.abs(C[i13, i12].astype(np.float64) - ref) / denom
            worst = max(worst, float(err.max()))
            if exact:
                avx = ORACLE.mul_mat_avx(t0, M, N, K, a, b)
                exact = bool(np.array_equal(avx.view(np.uint32), np.ascontiguousarray(C[i13, i12]).view(np.uint32)))
    return worst, exact


def _one(args):
    d, ent = args
    return (ent["phase"], layer_of(ent["src0"]), node_kind(ent["src0"]), ent["name"],
            (ent["ne0"][1], ent["ne1"][1], ent["ne0"][0], ent["ne0"][2])) + check_node(d, ent)


def check_nodes(d, workers=8):
    """[(phase, layer, kind, name, (M, N, K, slices), worst error, bit-exact in the reference's x86
    order (None: no restatement for the type))] for every dumped node, the
    nodes spread over `workers` processes (each loads its own oracle)"""
    with open(os.path.join(d, "index.jsonl")) as f:
        ents = [json.loads(line) for line in f]
    if workers <= 1:
        return [_one((d, e)) for e in ents]
    import multiprocessing as mp
    with mp.get_context("spawn").Pool(min(workers, len(ents))) as pool:
        return pool.map(_one, [(d, e) for e in ents], chunksize=1)
