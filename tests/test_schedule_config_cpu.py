"""CPU test of the schedule switches' lifetime (no GPU, no device call).

The switches that change which collectives an op posts (BAGUA_PIPELINE_PIECES,
BAGUA_PIPELINE_MIN_PIECE, BAGUA_PIPELINE_TAPER, BAGUA_RING_MULTIPATH,
BAGUA_CHECK_SCHEDULE) are read once, when a communicator is created
(comm_internal.hpp ScheduleConfig); an op never reads them again, so ranks cannot
drift apart mid-run.  Creating a loopback group and its communicators is pure host
code, so this runs anywhere the library loads: a child process sets the
environment, creates communicators, changes the environment, creates more, and
reports bagua_comm_schedule_config for each."""
import json
import os
import subprocess
import sys

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))

CHILD = r"""
import ctypes, json, os, sys
lib = ctypes.CDLL(os.path.join(sys.argv[1], "bagua-core_amd", "lib", "libbagua_core.so"))
lib.bagua_loopback_group_create.restype = ctypes.c_void_p
lib.bagua_loopback_group_create.argtypes = [ctypes.c_int, ctypes.c_int]
lib.bagua_loopback_communicator_create.restype = ctypes.c_void_p
lib.bagua_loopback_communicator_create.argtypes = [ctypes.c_void_p, ctypes.c_size_t, ctypes.c_uint64]
lib.bagua_comm_schedule_config.argtypes = [ctypes.c_void_p, ctypes.POINTER(ctypes.c_int32), ctypes.c_int]

def cfg(c):
    out = (ctypes.c_int32 * 5)()
    assert lib.bagua_comm_schedule_config(c, out, 5) == 0
    return list(out)

def comms(p):
    g = lib.bagua_loopback_group_create(p, 0)
    return [lib.bagua_loopback_communicator_create(g, r, 0) for r in range(p)]

res = {}
first = comms(2)
res["first"] = [cfg(c) for c in first]
os.environ.update({"BAGUA_PIPELINE_PIECES": "8", "BAGUA_PIPELINE_MIN_PIECE": "4096", "BAGUA_PIPELINE_TAPER": "1",
                   "BAGUA_RING_MULTIPATH": "1", "BAGUA_CHECK_SCHEDULE": "1"})
res["first_after_env_change"] = [cfg(c) for c in first]
res["second"] = [cfg(c) for c in comms(3)]
out = (ctypes.c_int32 * 5)()
res["too_small"] = lib.bagua_comm_schedule_config(first[0], out, 4)
res["null"] = lib.bagua_comm_schedule_config(None, out, 5)
print(json.dumps(res))
"""


def test_schedule_switches_are_fixed_at_creation():
    env = {k: v for k, v in os.environ.items()
           if k not in ("BAGUA_PIPELINE_PIECES", "BAGUA_PIPELINE_MIN_PIECE", "BAGUA_PIPELINE_TAPER",
                        "BAGUA_RING_MULTIPATH", "BAGUA_CHECK_SCHEDULE")}
    if not os.path.exists(os.path.join(ROOT, "bagua-core_amd", "lib", "libbagua_core.so")):
        pytest.skip("libbagua_core.so not built")
    r = subprocess.run([sys.executable, "-c", CHILD, ROOT], env=env, capture_output=True, text=True, timeout=120)
    assert r.returncode == 0, r.stderr[-2000:]
    res = json.loads(r.stdout.strip().splitlines()[-1])
    default = [4, 1 << 20, -1, 0, 0]  # taper -1: automatic piece schedules tapered
    assert res["first"] == [default, default]
    assert res["first_after_env_change"] == [default, default]  # fixed at creation
    assert res["second"] == [[8, 4096, 1, 1, 1]] * 3             # later communicators see the new values
    assert res["too_small"] != 0 and res["null"] != 0
