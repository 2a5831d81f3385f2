"""Config 4 at BASELINE.json's full size, checked through size-independent
properties (the oracle simulation of 8 ranks x 1 GiB would take minutes of CPU
time): p = 2, 4 or 8 virtual ranks on the loopback transport each own a 1 GiB
fp32 gradient (2^28 elements, p chunks of 2^28 / p), run the default
(pipelined, fused) compressed all-reduce, and then

  * every rank holds the same bytes (the allgather's guarantee), and
  * each element is within the format's two-quantisation bound of the exact
    mean of the 8 inputs: |y - mean| <= d1/2 + d2/2 (+ slack), where d1 is the
    widest per-rank step (max - min + 1e-7)/255 of that chunk and d2 the step of
    the reduced chunk (DESIGN.md §3 tolerance, applied twice).

A chunk routed to the wrong rank or reduced in the wrong slot lands ~1e-3 off
(the inputs' scale), ~25x outside the bound."""
import ctypes

import pytest
import torch

from test_gpu_multirank import run_ranks

pytestmark = pytest.mark.gpu


@pytest.mark.parametrize("p", [2, 4, 8])
def test_centralized_allreduce_1gib_properties(p):
    """Config 4 at 2, 4 and 8 ranks, 1 GiB fp32 per rank (every point of the 1/2/4/8 curve)."""
    import bagua_core
    from bagua_core.communicator import loopback_communicators
    N = bagua_core._native
    n = 1 << 28
    cs = n // p
    xs = []
    for r in range(p):
        g = torch.Generator(device="cuda").manual_seed(0x5EED + r)
        xs.append(torch.randn(n, device="cuda", generator=g) * 1e-3 + 1e-3 * r)
    mean = torch.zeros(n, dtype=torch.float64, device="cuda")
    for x in xs:
        mean += x.double()
    mean /= p
    # widest per-rank quantisation step of every chunk
    d1 = torch.zeros(p, dtype=torch.float64, device="cuda")
    for x in xs:
        c = x.view(p, cs)
        d1 = torch.maximum(d1, ((c.amax(1) - c.amin(1)).double() + 1e-7) / 255.0)
    comms = loopback_communicators(p, 0)
    torch.cuda.synchronize()

    def rank(r):
        raw = bagua_core.BaguaTensorPy(xs[r], f"g{r}").raw()
        N.check(N.C.bagua_centralized_low_precision_synchronous(comms[r].handle, ctypes.byref(raw), 1,
                                                                N.COMPRESSION_MINMAX_UINT8), f"rank {r}")

    run_ranks(rank, p)
    torch.cuda.synchronize()
    for r in range(1, p):
        assert torch.equal(xs[r].view(torch.int32), xs[0].view(torch.int32)), f"rank {r} differs from rank 0"
    y = xs[0].view(p, cs)
    d2 = ((y.amax(1) - y.amin(1)).double() + 2 * d1 + 1e-7) / 255.0
    bound = (0.5 * d1 + 0.5 * d2) * (1 + 1e-4) + 1e-9
    err = (y.double() - mean.view(p, cs)).abs().amax(1)
    assert bool((err <= bound).all()), f"max error per chunk {err.tolist()} vs bound {bound.tolist()}"
    # the bound is tight enough to mean something: far below the inputs' scale
    assert float(bound.max()) < 1e-4


def test_centralized_onebit_allreduce_1gib_p8_properties():
    """The same at full size with the 1-bit codec: ranks identical; inside every
    chunk each element is +-one scale; its sign is the sign of the exact mean m of
    the 8 decoded inputs (sign(x_r) * mean|x_r| per chunk) wherever |m| is not
    within rounding of 0; the scale is mean|m| of the chunk to f32 rounding of the
    tree sum (1e-5 relative)."""
    import bagua_core
    from bagua_core.communicator import loopback_communicators
    N = bagua_core._native
    p, n = 8, 1 << 28
    cs = n // p
    xs = []
    for r in range(p):
        g = torch.Generator(device="cuda").manual_seed(0x0B17 + r)
        xs.append(torch.randn(n, device="cuda", generator=g) * 1e-3)
    m = torch.zeros(p, cs, dtype=torch.float64, device="cuda")
    for x in xs:
        c = x.view(p, cs).double()
        m += torch.where(c < 0, -1.0, 1.0) * c.abs().mean(1, keepdim=True)
    m /= p
    comms = loopback_communicators(p, 0)
    torch.cuda.synchronize()

    def rank(r):
        raw = bagua_core.BaguaTensorPy(xs[r], f"g{r}").raw()
        N.check(N.C.bagua_centralized_low_precision_synchronous(comms[r].handle, ctypes.byref(raw), 1,
                                                                N.COMPRESSION_ONEBIT), f"rank {r}")

    run_ranks(rank, p)
    torch.cuda.synchronize()
    for r in range(1, p):
        assert torch.equal(xs[r].view(torch.int32), xs[0].view(torch.int32)), f"rank {r} differs from rank 0"
    y = xs[0].view(p, cs).double()
    scale = y.abs().amax(1)
    assert torch.equal(y.abs().amin(1), scale), "every element of a chunk is +-one scale"
    want_scale = m.abs().mean(1)
    assert bool(((scale - want_scale).abs() <= 1e-5 * want_scale).all()), (scale.tolist(), want_scale.tolist())
    clear = m.abs() > 1e-6 * m.abs().amax()
    assert bool((torch.sign(y)[clear] == torch.sign(m)[clear]).all()), "sign of the reduced mean"


@pytest.mark.parametrize("multipath", ["0", "1"])
def test_decentralized_ring_bf16_p8_full_size_properties(multipath, monkeypatch):
    """Config 5 at full size (2^27 bf16 elements per rank, 8 ranks; the default direct
    exchange and the opt-in multipath one): with mix_r = t_r + (l_r + r_r) f13 + w_r f53 (f13, f53 =
    1/3 and -5/3 rounded to bf16 as the 16-bit addmul does; the bucket
    each rank quantises, decentralized_low_precision_synchronous.rs:45-64) and
    d_r its quantisation step, after the op
      w_r' == t_r'                                   (:150-151 clone, exact)
      t_r' - w_r  ~ mix_r       within d_r/2          (own payload, :140-149)
      l_r' - l_r  ~ mix_{r-1}   within d_{r-1}/2      (left peer's payload, :126-131)
      r_r' - r_r  ~ mix_{r+1}   within d_{r+1}/2      (right peer's payload, :133-138)
    plus bf16 rounding of every stored step.  A payload from the wrong peer is
    ~1e-3 off, far outside."""
    import bagua_core
    from bagua_core.communicator import loopback_communicators
    N = bagua_core._native
    p, n = 8, 1 << 27
    ts = {k: [] for k in "twlr"}
    for r in range(p):
        g = torch.Generator(device="cuda").manual_seed(0xC0F5 + r)
        for k in "twlr":
            ts[k].append((torch.randn(n, device="cuda", generator=g) * 1e-3).to(torch.bfloat16))
    old = {k: [t.double() for t in ts[k]] for k in "wlr"}
    # 16-bit addmul multiplies by the factor rounded to T (K:83-91: __hmul(b, half(factor)))
    f13 = float(torch.tensor(1.0 / 3.0).to(torch.bfloat16))
    f53 = float(torch.tensor(-5.0 / 3.0).to(torch.bfloat16))
    mix = [ts["t"][r].double() + old["l"][r] * f13 + old["r"][r] * f13 + old["w"][r] * f53 for r in range(p)]
    # magnitude the mix's three rounded bf16 steps round at, per element
    mag = [ts["t"][r].double().abs() + old["l"][r].abs() / 3 + old["r"][r].abs() / 3 + 5 * old["w"][r].abs() / 3
           for r in range(p)]
    step = [float((mx.max() - mx.min()) + 1e-7) / 255.0 for mx in mix]
    monkeypatch.setenv("BAGUA_RING_MULTIPATH", multipath)  # read when the communicators are created
    comms = loopback_communicators(p, 0)
    torch.cuda.synchronize()

    def rank(r):
        raws = [bagua_core.BaguaTensorPy(ts[k][r], k).raw() for k in "twlr"]
        N.check(N.C.bagua_decentralized_low_precision_synchronous(comms[r].handle, *[ctypes.byref(x) for x in raws],
                                                                  N.COMPRESSION_MINMAX_UINT8), f"rank {r}")

    run_ranks(rank, p)
    torch.cuda.synchronize()
    for r in range(p):
        t_new = ts["t"][r].double()
        assert torch.equal(ts["w"][r].view(torch.int16), ts["t"][r].view(torch.int16)), f"rank {r}: w != t"
        for new_val, base, src in ((t_new, old["w"][r], r), (ts["l"][r].double(), old["l"][r], (r - 1) % p),
                                   (ts["r"][r].double(), old["r"][r], (r + 1) % p)):
            got = new_val - base
            # bf16 rounding, half an ulp = 2^-9 relative, element by element: the mix rounds
            # 6 times (3 products, 3 sums, each <= mag in size; 4 * mag covers them), the
            # decoded value once and the stored sum once (doubled for safety)
            bound = step[src] / 2 * (1 + 1e-4) + 2.0 ** -9 * (4 * mag[src] + 2 * got.abs() + 2 * new_val.abs())
            excess = float((( got - mix[src]).abs() - bound).max())
            assert excess <= 0, (r, src, excess, step[src])
