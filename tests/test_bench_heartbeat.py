"""bench.py's rank-0 heartbeat: progress lines go to stderr while a long run
(C5 at N = 2: minutes per run) renders, never to stdout (one JSON line)."""
from __future__ import annotations

import os
import sys
import time

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))

import bench  # noqa: E402


def test_heartbeat_writes_stderr_only(capsys):
    hb = bench.Heartbeat(True, period=0.05)
    hb.phase = "20 timed steps"
    time.sleep(0.3)
    hb.stop()
    time.sleep(0.1)
    out, err = capsys.readouterr()
    assert out == ""
    assert "bench: 20 timed steps (" in err
    n = err.count("\n")
    time.sleep(0.2)
    assert capsys.readouterr().err.count("\n") == 0 and n >= 2  # stopped


def test_heartbeat_disabled_on_other_ranks(capsys):
    hb = bench.Heartbeat(False, period=0.05)
    time.sleep(0.2)
    hb.stop()
    assert capsys.readouterr() == ("", "")
