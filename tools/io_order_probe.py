"""Measurement aid: does deleting a large tree slow the next writes on this filesystem?  Replays 118k files of ~31 KB
(config 2's cluster<N> shape) with tools/io_probe.c io_probe_replay three times: fresh, right after deleting the
previous replay's files, and after a pause.  Prints seconds and `df` of $TMPDIR."""
import ctypes
import os
import shutil
import subprocess
import sys
import tempfile
import time

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
from bench import replay_probe  # noqa: E402

d = tempfile.mkdtemp(prefix="ioorder_", dir=os.environ.get("TMPDIR", "/tmp"))
print(subprocess.run(["df", "-h", d], capture_output=True, text=True).stdout, flush=True)
print(subprocess.run(["stat", "-f", "-c", "%T", d], capture_output=True, text=True).stdout, flush=True)
sizes = list(np.random.default_rng(1).integers(20000, 42000, size=118000))
T = int(sys.argv[1]) if len(sys.argv) > 1 else 16
try:
    def keep(tag):  # a replay whose files stay (io_probe_replay removes them itself; time the removal separately)
        t0 = time.perf_counter()
        r = replay_probe(d, sizes, 50_000_000, T)
        return r["seconds"], time.perf_counter() - t0
    print("fresh", keep("a"), flush=True)
    os.sync()
    print("after delete+sync", keep("b"), flush=True)
    time.sleep(20)
    print("after 20 s pause", keep("c"), flush=True)
    os.sync()
    time.sleep(5)
    print("after sync + 5 s", keep("d"), flush=True)
finally:
    shutil.rmtree(d, ignore_errors=True)
