#!/usr/bin/env python3
"""Per-rank codec kernels of the pipelined MinMax op (comm_ops.cpp centralized_pipelined)
at p = 2, 4, 8 on a 1 GiB fp32 bucket, timed one by one on one GPU with the kernels'
own HIP events (bagua_time_next_kernel), without the exchange: what the §6 prediction
of the N > 1 step needs -- the prefix before the first alltoall piece (min/max pass +
quantise of piece 0), the middle between the last alltoall and the first allgather
piece (reduce of the last piece + requantise of piece 0), the suffix after the last
allgather piece (dequantise of the last piece), and the total codec time per op.

    python tools/pipeline_kernels_probe.py [--pieces 4] [--reps 5] [--onebit-only] [--log2n 28]
"""
import argparse
import ctypes
import json
import os
import sys

import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "bagua-core_amd"))


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--pieces", type=int, default=4)
    ap.add_argument("--reps", type=int, default=5)
    ap.add_argument("--tapered", action="store_true", help="first and last piece half size (PIECES_TAPERED)")
    ap.add_argument("--no-tables", action="store_true",
                    help="every reduce / requantise piece builds its own tables (the op copies piece 0's)")
    ap.add_argument("--onebit-only", action="store_true", help="the 1-bit op's kernels only")
    ap.add_argument("--log2n", type=int, default=28, help="bucket elements (fp32), log2")
    a = ap.parse_args()
    from bagua_core import _native as N
    K = N.K
    dev = torch.device("cuda", 0)
    n = 1 << a.log2n
    g = torch.Generator(device=dev).manual_seed(3)
    x = torch.randn(n, device=dev, generator=g) * 1e-3
    st = torch.cuda.current_stream()
    sp = ctypes.c_void_p(st.cuda_stream)
    out = {"bucket_bytes": 4 * n, "pieces": a.pieces, "tapered": a.tapered, "tables": not a.no_tables}

    def timed(call):
        ts = []
        for _ in range(a.reps):
            e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
            e0.record(st)
            e1.record(st)
            N.check(K.bagua_time_next_kernel(e0.cuda_event, e1.cuda_event), "timing hook")
            N.check(call(), "kernel")
            torch.cuda.synchronize()
            ts.append(e0.elapsed_time(e1) * 1e3)
        ts.sort()
        return ts[len(ts) // 2]

    for p in (() if a.onebit_only else (2, 4, 8)):
        cs = n // p
        P = a.pieces
        SCH = P | (N.PIECES_TAPERED if a.tapered else 0)  # the piece schedule every piece call takes
        if not a.no_tables:  # as the op: reduce piece 0 leaves its tables, the later pieces copy them
            SCH |= N.PIECES_TABLES
        S = K.bagua_minmax_u8_compressed_bytes(0, cs, p)
        wsb = max(K.bagua_minmax_u8_workspace_bytes(cs, p), K.bagua_minmax_u8_pipeline_workspace_bytes(cs, SCH))
        send = torch.empty(S, dtype=torch.uint8, device=dev)
        ws = torch.empty(wsb, dtype=torch.uint8, device=dev)
        xp, cp, wp = x.data_ptr(), send.data_ptr(), ws.data_ptr()
        r = p - 1

        def rng(q):
            b, e = ctypes.c_int(), ctypes.c_int()
            N.check(K.bagua_minmax_u8_piece_range(cs, SCH, q, ctypes.byref(b), ctypes.byref(e)), "range")
            return b.value, e.value
        row = {}
        row["minmax_pass_us"] = timed(lambda: K.bagua_minmax_u8_compress_stage(5, 0, xp, n, cs, p, cp, S, wp, wsb, -1,
                                                                                sp))
        q_us = [timed(lambda q=q: K.bagua_minmax_u8_quantize_range(0, xp, n, cs, p, cp, S, wp, wsb, -1, *rng(q), sp))
                for q in range(P)]
        # the received buffer: a second copy of this rank's compressed bytes stands in for the
        # peers' (its own segments differ from the ones it sends, as on a node)
        recv = send.clone()
        rp = recv.data_ptr()
        # storing pair (BAGUA_PIPE_RECOMPUTE=0): the reduce piece stores the reduced piece of
        # the own chunk (4 B per element) and the requantise reads it back
        r_us = [timed(lambda q=q: K.bagua_minmax_u8_reduce_piece(0, rp, S, cs, p, xp, 1, r, SCH, q, wp, wsb, sp))
                for q in range(P)]
        rq_us = [timed(lambda q=q: K.bagua_minmax_u8_requantize_piece(0, xp, cs, p, cp, S, r, SCH, q, wp, wsb, sp))
                 for q in range(P)]
        # the op's default: partials-only reduce pieces, the requantise recomputes from recv
        r2_us = [timed(lambda q=q: K.bagua_minmax_u8_reduce_piece(0, rp, S, cs, p, None, 1, r, SCH, q, wp, wsb, sp))
                 for q in range(P)]
        rq2_us = [timed(lambda q=q: K.bagua_minmax_u8_reduce_requantize_piece(0, rp, S, cs, p, 1, cp, S, r, SCH, q, wp,
                                                                              wsb, sp))
                  for q in range(P)]
        d_us = [timed(lambda q=q: K.bagua_minmax_u8_decompress_range(0, cp, S, cs, p, xp, *rng(q), sp))
                for q in range(P)]
        r1 = lambda v: [round(u, 1) for u in v]
        row.update({"quantise_piece_us": r1(q_us), "dequantise_piece_us": r1(d_us),
                    "store": {"reduce_piece_us": r1(r_us), "requantise_piece_us": r1(rq_us)},
                    "recompute": {"reduce_piece_us": r1(r2_us), "requantise_piece_us": r1(rq2_us)}})
        # algorithmic bytes per launch: piece q covers L_q elements of every chunk
        L = [rng(q)[1] - rng(q)[0] for q in range(P)]
        rate = lambda byts, us: round(byts / us / 1e3, 1)  # GB/s
        row["minmax_pass_gb_s"] = rate(4 * n, row["minmax_pass_us"])              # x read once
        row["quantise_piece_gb_s"] = [rate(5 * p * L[q], q_us[q]) for q in range(P)]  # x read, payload written
        row["dequantise_piece_gb_s"] = [rate(5 * p * L[q], d_us[q]) for q in range(P)]  # p payloads read, x written
        # storing pair: reduce = p payloads read + the fp32 piece written; requantise = that piece
        # read back + its payload written
        row["store"]["reduce_piece_gb_s"] = [rate((p + 4) * L[q], r_us[q]) for q in range(P)]
        row["store"]["requantise_piece_gb_s"] = [rate(5 * L[q], rq_us[q]) for q in range(P)]
        # recompute: reduce = p payloads read; requantise = p payloads read + its payload written
        row["recompute"]["reduce_piece_gb_s"] = [rate(p * L[q], r2_us[q]) for q in range(P)]
        row["recompute"]["requantise_piece_gb_s"] = [rate((p + 1) * L[q], rq2_us[q]) for q in range(P)]
        row["prefix_us"] = round(row["minmax_pass_us"] + q_us[0], 1)
        row["store"]["middle_us"] = round(r_us[-1] + rq_us[0], 1)
        row["recompute"]["middle_us"] = round(r2_us[-1] + rq2_us[0], 1)
        # the op's order since round 6: the LAST piece is requantised (and gathered) first,
        # right after its reduce, while its bytes are still in the caches
        # In the op the requantise follows the reduce pieces, not itself: time it (and the
        # last reduce piece) in that order from a flushed Infinity Cache, requantising piece
        # 0 first (round 5's order) or the last piece first (round 6's)
        flush = torch.empty(1 << 29, dtype=torch.uint8, device=dev)

        def in_order(store, first, prefold=False):
            ts = []
            for _ in range(a.reps):
                flush.add_(1)  # 512 MiB read + written: the caches hold nothing of this op
                for q in range(P - 1):
                    K.bagua_minmax_u8_reduce_piece(0, rp, S, cs, p, xp if store else None, 1, r, SCH, q, wp, wsb, sp)
                e = [torch.cuda.Event(enable_timing=True) for _ in range(6)]
                for ev in e:
                    ev.record(st)
                N.check(K.bagua_time_next_kernel(e[0].cuda_event, e[1].cuda_event), "timing hook")
                K.bagua_minmax_u8_reduce_piece(0, rp, S, cs, p, xp if store else None, 1, r, SCH, P - 1, wp, wsb, sp)
                rs = SCH
                if prefold:  # one workgroup folds every piece's partials; the requantise reads one value
                    N.check(K.bagua_time_next_kernel(e[4].cuda_event, e[5].cuda_event), "timing hook")
                    N.check(K.bagua_minmax_u8_fold_piece_partials(0, cs, SCH, wp, wsb, sp), "fold")
                    rs = SCH | N.PIECES_FOLDED
                N.check(K.bagua_time_next_kernel(e[2].cuda_event, e[3].cuda_event), "timing hook")
                if store:
                    N.check(K.bagua_minmax_u8_requantize_piece(0, xp, cs, p, cp, S, r, rs, first, wp, wsb, sp), "rq")
                else:
                    N.check(K.bagua_minmax_u8_reduce_requantize_piece(0, rp, S, cs, p, 1, cp, S, r, rs, first, wp,
                                                                      wsb, sp), "rrq")
                torch.cuda.synchronize()
                t = e[0].elapsed_time(e[1]) + e[2].elapsed_time(e[3]) + (e[4].elapsed_time(e[5]) if prefold else 0)
                ts.append(t * 1e3)
            ts.sort()
            return round(ts[len(ts) // 2], 1)
        for m, store in (("store", True), ("recompute", False)):
            row[m]["middle_in_order_first_piece_us"] = in_order(store, 0)
            row[m]["middle_in_order_last_piece_us"] = in_order(store, P - 1)
            row[m]["middle_in_order_prefold_us"] = in_order(store, 0, prefold=True)
        del flush
        row["suffix_us"] = round(d_us[-1], 1)
        common = row["minmax_pass_us"] + sum(q_us) + sum(d_us)
        row["store"]["codec_total_us"] = round(common + sum(r_us) + sum(rq_us), 1)
        row["recompute"]["codec_total_us"] = round(common + sum(r2_us) + sum(rq2_us), 1)
        # the recompute requantise writes the same bytes as the storing pair
        K.bagua_minmax_u8_reduce_piece(0, rp, S, cs, p, xp, 1, r, SCH, 0, wp, wsb, sp)
        for q in range(P):
            K.bagua_minmax_u8_reduce_piece(0, rp, S, cs, p, xp, 1, r, SCH, q, wp, wsb, sp)
        for q in range(P):
            K.bagua_minmax_u8_requantize_piece(0, xp, cs, p, cp, S, r, SCH, q, wp, wsb, sp)
        snap = send.clone()
        for q in range(P):
            K.bagua_minmax_u8_reduce_piece(0, rp, S, cs, p, None, 1, r, SCH, q, wp, wsb, sp)
        for q in range(P):
            K.bagua_minmax_u8_reduce_requantize_piece(0, rp, S, cs, p, 1, cp, S, r, SCH, q, wp, wsb, sp)
        torch.cuda.synchronize()
        row["recompute_bytes_equal"] = bool(torch.equal(snap, send))
        N.check(K.bagua_minmax_u8_fold_piece_partials(0, cs, SCH, wp, wsb, sp), "fold")
        for q in range(P):
            K.bagua_minmax_u8_reduce_requantize_piece(0, rp, S, cs, p, 1, cp, S, r, SCH | N.PIECES_FOLDED, q, wp, wsb,
                                                      sp)
        torch.cuda.synchronize()
        row["prefold_bytes_equal"] = bool(torch.equal(snap, send))
        del recv
        row["minmax_pass_us"] = round(row["minmax_pass_us"], 1)
        out[f"p{p}"] = row
        del send, ws
    # the 1-bit op (centralized_pipelined_onebit): encode pieces, finalize, fused middle
    # step (decode p segments + reduce + re-encode + finalize), decode pieces
    for p in (2, 4, 8):
        cs = n // p
        P = a.pieces
        S = K.bagua_onebit_compressed_bytes(cs, p)
        wsb = K.bagua_onebit_workspace_bytes(cs, p)
        send = torch.empty(S, dtype=torch.uint8, device=dev)
        res = torch.empty(S, dtype=torch.uint8, device=dev)
        ws = torch.empty(wsb, dtype=torch.uint8, device=dev)
        xp, cp, rp, wp = x.data_ptr(), send.data_ptr(), res.data_ptr(), ws.data_ptr()

        def trng(q):
            b, e = ctypes.c_int(), ctypes.c_int()
            N.check(K.bagua_onebit_piece_range(cs, P, q, ctypes.byref(b), ctypes.byref(e)), "range")
            return b.value, e.value
        e_us = [timed(lambda q=q: K.bagua_onebit_encode_range(0, xp, n, cs, p, cp, S, wp, wsb, *trng(q), sp))
                for q in range(P)]
        f_us = timed(lambda: K.bagua_onebit_finalize(wp, wsb, n, cs, p, cp, S, sp))
        m_us = timed(lambda: K.bagua_onebit_reduce_requantize(0, cp, S, cs, p, None, 1, rp, S, p - 1, wp, wsb, sp))
        # the whole middle call (its table kernel and the own segment's finalize), events around it
        mc = []
        for _ in range(a.reps):
            e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
            e0.record(st)
            N.check(K.bagua_onebit_reduce_requantize(0, cp, S, cs, p, None, 1, rp, S, p - 1, wp, wsb, sp), "middle")
            e1.record(st)
            torch.cuda.synchronize()
            mc.append(e0.elapsed_time(e1) * 1e3)
        mc.sort()
        d_us = [timed(lambda q=q: K.bagua_onebit_decompress_range(0, cp, S, cs, p, xp, *trng(q), sp))
                for q in range(P)]
        TL = [trng(q)[1] - trng(q)[0] for q in range(P)]  # tiles of 1024 elements per chunk
        out[f"onebit_p{p}_gb_s"] = {
            "encode_piece": [round(p * t * (4096 + 128) / us / 1e3, 1) for t, us in zip(TL, e_us)],
            "decode_piece": [round(p * t * (4096 + 128) / us / 1e3, 1) for t, us in zip(TL, d_us)],
            "middle": round((p + 1) * sum(TL) * 128 / m_us / 1e3, 1)}
        out[f"onebit_p{p}"] = {"encode_piece_us": [round(v, 1) for v in e_us], "finalize_us": round(f_us, 1),
                               "middle_us": round(m_us, 1), "middle_call_us": round(mc[len(mc) // 2], 1),
                               "decode_piece_us": [round(v, 1) for v in d_us],
                               "codec_total_us": round(sum(e_us) + f_us + m_us + sum(d_us), 1)}
        del send, res, ws
    print(json.dumps(out), flush=True)


if __name__ == "__main__":
    main()
