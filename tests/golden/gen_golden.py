"""Generate the committed golden fixtures tests/golden/codec_v1.npz.

The reference ships no golden vectors for this path and cannot be built or
imported here, so the fixtures are produced by the C
restatement (oracle/bagua_oracle.c) and accepted only if the independently
written numpy restatement (oracle/oracle_np.py) reproduces every byte.
Inputs are seeded numpy draws; the cases follow SURVEY.md §8(c): N(0, s^2)
for s in {1e-8, 1e-3, 1, 1e3}, offset means, all-equal, all-zero, +-0 mixes,
denormals, NaN/Inf, p in {1,2,3,4,8}, ragged chunk sizes, target chunks.

Run:  python tests/golden/gen_golden.py
"""
from __future__ import annotations

import os
import sys

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path.insert(0, ROOT)

from oracle import oracle_c as C  # noqa: E402
from oracle import oracle_np as NP  # noqa: E402
from oracle import simulate  # noqa: E402

KINDS = ["n1e-3", "n1e-8", "n1", "n1e3", "offset", "const", "zeros", "signed_zeros", "denormal", "nan", "inf"]
DTYPES = [C.F32, C.F16, C.BF16]
OUT = os.path.join(os.path.dirname(os.path.abspath(__file__)), "codec_v1.npz")


def make_input(kind: str, n: int, dtype: int, rng: np.random.Generator) -> np.ndarray:
    z = rng.standard_normal(n).astype(np.float32)
    if kind.startswith("n") and kind[1:].replace("e-", "").replace("e", "").isdigit():
        x = z * np.float32(float(kind[1:]))
    elif kind == "offset":
        x = z + np.float32(1e3 if dtype != C.F32 else 1e4)
    elif kind == "const":
        x = np.full(n, 0.37, np.float32)
    elif kind == "zeros":
        x = np.zeros(n, np.float32)
    elif kind == "signed_zeros":
        x = np.where(rng.random(n) < 0.5, np.float32(-0.0), np.float32(0.0)).astype(np.float32)
        x[::7] = z[::7] * np.float32(1e-3)
    elif kind == "denormal":
        x = z * np.float32(1e-39) if dtype != C.F16 else z * np.float32(1e-6)
    elif kind == "nan":
        x = z.copy()
        x[::13] = np.nan
    elif kind == "inf":
        x = z.copy()
        x[5::17] = np.inf
    else:
        raise ValueError(kind)
    if dtype == C.F32:
        return x.astype(np.float32)
    if dtype == C.F16:
        with np.errstate(over="ignore"):
            return x.astype(np.float16)
    return NP.from_f32(x, C.BF16)


def same_bytes(a: np.ndarray, b: np.ndarray) -> bool:
    return a.shape == b.shape and a.view(np.uint8).tobytes() == b.view(np.uint8).tobytes()


def main() -> None:
    rng = np.random.default_rng(0x5EED)
    out: dict[str, np.ndarray] = {}
    case = 0
    shapes = [(1, 1), (1, 7), (1, 4099), (2, 1000), (3, 517), (4, 1024), (8, 333)]
    # ---- MinMax-UInt8 compress / decompress (+ target chunk) ------------------
    for dtype in DTYPES:
        for ki, kind in enumerate(KINDS):
            p, cs = shapes[(ki + dtype) % len(shapes)]
            x = make_input(kind, p * cs, dtype, rng)
            for target in ([-1] if p == 1 else [-1, p - 1]):
                comp = C.compress_minmax_u8(x, dtype, p, target)
                assert same_bytes(comp, NP.compress_minmax_u8(x, dtype, p, target)), ("minmax", kind, dtype)
                dec = np.zeros_like(x)
                if target == -1:
                    C.decompress_minmax_u8(comp, p, dec, dtype)
                    dn = np.zeros_like(x)
                    NP.decompress_minmax_u8(comp, p, dn, dtype)
                    assert same_bytes(dec, dn), ("decompress", kind, dtype)
                out[f"mm_in_{case}"] = x.view(np.uint8)
                out[f"mm_meta_{case}"] = np.array([dtype, p, cs, target, ki], np.int64)
                out[f"mm_comp_{case}"] = comp
                out[f"mm_dec_{case}"] = dec.view(np.uint8)
                case += 1
    # ---- chunk reduction ---------------------------------------------------------
    rcase = 0
    for dtype in DTYPES:
        for p in (1, 2, 3, 4, 5, 8, 9, 16, 17, 33):
            cs = int(rng.integers(1, 300))
            x = make_input("n1", p * cs, dtype, rng)
            target = int(rng.integers(0, p))
            for avg in (0, 1):
                a = x.copy()
                C.reduce_chunks(a, dtype, p, target, avg)
                b = x.copy()
                NP.reduce_chunks(b, dtype, p, target, avg)
                assert same_bytes(a, b), ("reduce", p, dtype)
                out[f"red_in_{rcase}"] = x.view(np.uint8)
                out[f"red_meta_{rcase}"] = np.array([dtype, p, cs, target, avg], np.int64)
                out[f"red_out_{rcase}"] = a.view(np.uint8)
                rcase += 1
    # ---- 1-bit sign + scale --------------------------------------------------------
    ocase = 0
    for dtype in DTYPES:
        for p, cs in [(1, 1), (1, 1023), (1, 1025), (2, 4096), (3, 2000), (1, 1024 * 1024 + 5)]:
            x = make_input("n1e-3", p * cs, dtype, rng)
            comp = C.compress_onebit(x, dtype, p, -1)
            assert same_bytes(comp, NP.compress_onebit(x, dtype, p, -1)), ("onebit", p, cs, dtype)
            dec = np.zeros_like(x)
            C.decompress_onebit(comp, p, dec, dtype)
            dn = np.zeros_like(x)
            NP.decompress_onebit(comp, p, dn, dtype)
            assert same_bytes(dec, dn)
            if cs > 100000:  # keep the fixture small: store only the header + a hash of the big case
                out[f"ob_bigsum_{ocase}"] = np.frombuffer(comp[:32].tobytes(), np.uint8)
            out[f"ob_in_{ocase}"] = x.view(np.uint8) if cs <= 100000 else np.zeros(0, np.uint8)
            out[f"ob_meta_{ocase}"] = np.array([dtype, p, cs, 0], np.int64)
            out[f"ob_comp_{ocase}"] = comp if cs <= 100000 else comp[:32]
            out[f"ob_dec_{ocase}"] = dec.view(np.uint8) if cs <= 100000 else np.zeros(0, np.uint8)
            ocase += 1
    # ---- op simulations (centralized, decentralized) ---------------------------------
    scase = 0
    for dtype in (C.F32, C.BF16):
        for p, cs in [(1, 1 << 12), (2, 1000), (4, 999), (8, 512)]:
            xs = [make_input("n1e-3", p * cs, dtype, rng) for _ in range(p)]
            if (C.minmax_compressed_size(p, cs, dtype)) % p:
                continue
            ya = simulate.centralized_low_precision(C, xs, dtype, True)
            yb = simulate.centralized_low_precision(NP, xs, dtype, True)
            assert all(same_bytes(a, b) for a, b in zip(ya, yb)), ("centralized", p, dtype)
            assert all(same_bytes(ya[0], y) for y in ya), "all ranks must end identical"
            out[f"cen_meta_{scase}"] = np.array([dtype, p, cs], np.int64)
            out[f"cen_in_{scase}"] = np.stack([x.view(np.uint8) for x in xs])
            out[f"cen_out_{scase}"] = ya[0].view(np.uint8)
            scase += 1
    dcase = 0
    for dtype in (C.F32, C.BF16, C.F16):
        for p, n in [(1, 777), (2, 1000), (3, 4099)]:
            ts = [make_input("n1e-3", n, dtype, rng) for _ in range(p)]
            ws = [make_input("n1e-3", n, dtype, rng) for _ in range(p)]
            ls = [make_input("n1e-3", n, dtype, rng) for _ in range(p)]
            rs = [make_input("n1e-3", n, dtype, rng) for _ in range(p)]
            ra = simulate.decentralized_low_precision(C, ts, ws, ls, rs, dtype)
            rb = simulate.decentralized_low_precision(NP, ts, ws, ls, rs, dtype)
            for ga, gb in zip(ra, rb):
                assert all(same_bytes(a, b) for a, b in zip(ga, gb)), ("decentralized", p, dtype)
            out[f"dec_meta_{dcase}"] = np.array([dtype, p, n], np.int64)
            for nm, arrs in zip(("t", "w", "l", "r"), (ts, ws, ls, rs)):
                out[f"dec_in_{nm}_{dcase}"] = np.stack([a.view(np.uint8) for a in arrs])
            for nm, arrs in zip(("t", "w", "l", "r"), ra):
                out[f"dec_out_{nm}_{dcase}"] = np.stack([a.view(np.uint8) for a in arrs])
            dcase += 1
    # ---- partially valid tensors: num_elements() < num_elements_allocated -----------------
    # K:538-545 limits each chunk's min/max to min(remaining, chunk_size) elements (an empty
    # range when remaining <= 0: header = init), while K:468-472 quantises every element of
    # every chunk with that chunk's parameters.  Both restatements must agree byte for byte.
    pcase = 0
    for dtype in DTYPES:
        for p, cs, n_in, target in [(4, 1000, 3 * 1000 + 321, -1),  # last chunk ragged
                                    (4, 1000, 2 * 1000, -1),        # last two chunks empty
                                    (3, 517, 5, -1),                # first chunk holds 5 elements
                                    (1, 4099, 0, -1),               # nothing valid at all
                                    (5, 203, 4 * 203 - 10, 3),      # ragged target chunk
                                    (5, 203, 4 * 203 - 10, 4),      # empty target chunk
                                    (2, 1000, 1500, -1)]:
            x = make_input("offset" if p == 2 else "n1e-3", p * cs, dtype, rng)
            comp = C.compress_minmax_u8(x, dtype, p, target, num_elem=n_in)
            assert same_bytes(comp, NP.compress_minmax_u8(x, dtype, p, target, num_elem=n_in)), \
                ("minmax partial", p, cs, n_in, target, dtype)
            dec = np.zeros_like(x)
            if target == -1:
                C.decompress_minmax_u8(comp, p, dec, dtype)
                dn = np.zeros_like(x)
                NP.decompress_minmax_u8(comp, p, dn, dtype)
                assert same_bytes(dec, dn), ("decompress partial", p, cs, dtype)
            out[f"mmp_in_{pcase}"] = x.view(np.uint8)
            out[f"mmp_meta_{pcase}"] = np.array([dtype, p, cs, target, n_in], np.int64)
            out[f"mmp_comp_{pcase}"] = comp
            out[f"mmp_dec_{pcase}"] = dec.view(np.uint8)
            pcase += 1
    cpcase = 0
    for dtype in (C.F32, C.BF16):
        for p, cs, short in [(2, 1000, 37), (4, 999, 500), (3, 512, 517)]:
            xs = [make_input("n1e-3", p * cs, dtype, rng) for _ in range(p)]
            if (C.minmax_compressed_size(p, cs, dtype)) % p:
                continue
            ya = simulate.centralized_low_precision(C, xs, dtype, True, num_elem=p * cs - short)
            yb = simulate.centralized_low_precision(NP, xs, dtype, True, num_elem=p * cs - short)
            assert all(same_bytes(a, b) for a, b in zip(ya, yb)), ("centralized partial", p, dtype)
            out[f"cenp_meta_{cpcase}"] = np.array([dtype, p, cs, p * cs - short], np.int64)
            out[f"cenp_in_{cpcase}"] = np.stack([x.view(np.uint8) for x in xs])
            out[f"cenp_out_{cpcase}"] = np.stack([y.view(np.uint8) for y in ya])
            cpcase += 1
    out["counts"] = np.array([case, rcase, ocase, scase, dcase, pcase, cpcase], np.int64)
    np.savez_compressed(OUT, **out)
    print(f"wrote {OUT}: minmax {case}, reduce {rcase}, onebit {ocase}, centralized {scase}, decentralized {dcase}, "
          f"partial minmax {pcase}, partial centralized {cpcase}; "
          f"{os.path.getsize(OUT)} bytes")


if __name__ == "__main__":
    main()
