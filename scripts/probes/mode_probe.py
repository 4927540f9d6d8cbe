"""Where does the S-K "slow mode" come from?  Some processes replay the same graph ~16 us (~4.6 %)
slower than others, for every build alike.  This probe times the replayed S-K graph in one process:
  1. on the default stream, several windows (is the mode stable within a process?);
  2. on fresh streams (normal and high priority): is it the hardware queue the stream maps to?
  3. after rebuilding the hot path (new buffers, new plan): is it where the buffers landed?

    python scripts/probes/mode_probe.py
"""
from __future__ import annotations

import os
import statistics
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path.insert(0, ROOT)
sys.path.insert(0, os.path.join(ROOT, "scripts"))

import torch  # noqa: E402

import step_tune  # noqa: E402


def window(hp, stream, reps: int) -> float:
    with torch.cuda.stream(stream):
        for _ in range(3):
            hp.launch(stream)
        a, b = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        a.record(stream)
        for _ in range(reps):
            hp.launch(stream)
        b.record(stream)
    b.synchronize()
    return a.elapsed_time(b) / reps * 1e3


def med(hp, stream, reps, n=7) -> str:
    ts = [window(hp, stream, reps) for _ in range(n)]
    return f"{statistics.median(ts):7.2f} us (min {min(ts):7.2f} max {max(ts):7.2f})"


def main():
    dev = torch.device("cuda", 0)
    torch.cuda.set_device(dev)
    hps = [step_tune.build("S", dev)]
    reps = step_tune.reps_for(hps[0])
    default = torch.cuda.current_stream(dev)
    print("default stream       ", med(hps[0], default, reps), flush=True)
    streams = [("new stream %d" % i, torch.cuda.Stream(dev)) for i in range(3)]
    streams += [("high-priority stream", torch.cuda.Stream(dev, priority=-1))]
    for name, st in streams:
        hps[0]._graph_ready = False  # rebuild the graph for the stream (capture is stream-independent)
        print(f"{name:21s}", med(hps[0], st, reps), flush=True)
    print("default stream again ", med(hps[0], default, reps), flush=True)
    for i in range(3):
        hps.append(step_tune.build("S", dev))
        print(f"rebuilt hot path {i}   ", med(hps[-1], default, reps), flush=True)
    print("first hot path again ", med(hps[0], default, reps), flush=True)
    for hp in hps:
        hp.close()


if __name__ == "__main__":
    main()
