"""The product library ignores the lab environment knobs (compiled in only with -DSDRG_LAB=1, tools/build_variant.sh):
a fresh process with SDRG_PIPE_SKIP (which skips SSB roles: wrong PCM in a lab build), SDRG_PIPE_MAP, SDRG_CU_SPLIT
and the other knobs set before any GPU call produces spectra, records and PCM bit-identical to a clean process."""
import os
import subprocess
import sys

import pytest

from conftest import ROOT

pytestmark = pytest.mark.gpu

KNOBS = {"SDRG_PIPE_SKIP": "0xfff", "SDRG_PIPE_MAP": "0", "SDRG_CU_SPLIT": "1", "SDRG_PIPE_PRIO": "0xfff",
         "SDRG_SSB_REFERENCE_KERNELS": "1", "SDRG_SPECTRUM_GRID": "3", "SDRG_STREAM_PRIO": "-1,1",
         "SDRG_EVENT_FENCE": "1", "SDRG_PIPE_STAMPS": "1", "SDRG_QUEUES": "31,1",
         "SDRG_GATHER_STREAM": "1", "SDRG_WIDE_SINGLE": "1", "SDRG_SSB_FIRST": "1", "SDRG_STATS_CUS": "32"}


def _run(extra):
    env = {k: v for k, v in os.environ.items() if not k.startswith("SDRG_")}
    env.update(extra)
    r = subprocess.run([sys.executable, os.path.join(ROOT, "tests", "lab_knob_child.py")], capture_output=True,
                       text=True, timeout=180, env=env)
    assert r.returncode == 0, r.stderr[-2000:]
    return r.stdout.strip().splitlines()[-1]


def test_lab_knobs_have_no_effect_on_the_product_library():
    clean = _run({})
    assert _run(KNOBS) == clean
