"""BASELINE configs[3]'s collective behind the C ABI: RCCL's ncclGather driven by libsdrg.so
itself (sdrg_dist_create + sdrg_engine_gather), in an interpreter that never imports torch, so a C/C++ host behind
the JNI boundary can shard and gather without PyTorch.  One rank (the box has one GPU; RCCL refuses two ranks on one
device), a pipelined engine with asynchronous statistics, four calls with their gathers and no host synchronisation
between them: the gathered records, focus slices, full spectra and PCM equal a joined engine's outputs bit for bit.
The per-frame payload is soapyCallback's (sdr-bridge-java-soapy.cpp:456-466) and the SSB worker's
(ssb_processor.cpp:103-108)."""
import json
import os
import subprocess
import sys

import pytest

from conftest import ROOT

pytestmark = pytest.mark.gpu


@pytest.mark.parametrize("mode", ["all", "nopcm", "sync"])
@pytest.mark.parametrize("rccl_one_rank", [True, False], ids=["rccl", "device_copies"])
def test_capi_rccl_gathers_equal_engine_outputs_without_torch(rccl_one_rank, mode):
    """rccl: sdrg_dist_set_one_rank_rccl(d, 1) keeps the one-rank gathers on RCCL's ncclGather (the N > 1 data path);
    device_copies: the one-rank default, hipMemcpyAsync (sdrg_dist_info reports which).  mode: which engine stream the
    gathers run on (all: with PCM, the audio detector's; nopcm: the asynchronous statistics'; sync: the main stream)."""
    worker = os.path.join(ROOT, "tests", "dist_capi_worker.py")
    env = dict(os.environ, PYTHONPATH="", DIST_CAPI_ONE_RANK_RCCL="1" if rccl_one_rank else "0", DIST_CAPI_MODE=mode)
    r = subprocess.run([sys.executable, "-u", worker], capture_output=True, text=True, timeout=240, env=env)
    assert r.returncode == 0, r.stderr[-4000:]
    line = [ln for ln in r.stdout.splitlines() if ln.startswith("{")][-1]
    res = json.loads(line)
    assert res["torch_loaded"] is False
    assert res["world"] == 1 and res["rccl_version"] > 0
    assert res["rccl_data"] is rccl_one_rank and res["mode"] == mode
    assert res["ok"] and all(res["ok"].values()), res["ok"]
