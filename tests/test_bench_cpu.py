"""CPU tests of bench.py's host-side legs: the cpu_baseline functions (the
reference algorithm = the C oracle on the host cores) and the
host description every line carries.  No GPU: small tensors on the CPU."""
import argparse
import os
import sys

import numpy as np
import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)

import bench  # noqa: E402


def _args(**kw):
    a = argparse.Namespace(cpu_seconds=0.05)
    for k, v in kw.items():
        setattr(a, k, v)
    return a


def test_host_info_fields():
    h = bench.host_info()
    assert h["os_cpu_count"] >= 1 and h["affinity_cpus"] >= 1
    assert "cpu_model" in h


def test_cpu_codec_baseline_same_bucket(oracle_c):
    x = torch.randn(1 << 16) * 1e-3
    comp = torch.from_numpy(oracle_c.compress_minmax_u8(x.numpy(), 0, 1))
    c = bench.cpu_codec_baseline(_args(), x, comp)
    assert c["kind"] == "port" and c["value"] > 0 and c["cores"] >= 1
    assert c["matches_gpu_bytes"] is True  # the given bytes are the oracle's own here
    assert "0 MiB bucket" in c["sample"] or "MiB bucket" in c["sample"]
    bad = comp.clone()
    bad[40] ^= 1
    assert bench.cpu_codec_baseline(_args(), x, bad)["matches_gpu_bytes"] is False


def test_cpu_codec_baseline_onebit_and_bf16(oracle_c):
    x = (torch.randn(1 << 15) * 1e-3).to(torch.bfloat16)
    c = bench.cpu_codec_baseline(_args(), x, None, onebit=True)
    assert c["value"] > 0 and c["matches_gpu_bytes"] is None and "1-bit" in c["sample"]


def test_cpu_allreduce_baseline_all_ranks(oracle_c):
    c = bench.cpu_allreduce_baseline(_args(), 4, 1 << 14, torch.device("cpu"), sample_elems=1 << 12)
    assert c["value"] > 0 and "4 ranks" in c["sample"] and c["host"]["os_cpu_count"] >= 1
