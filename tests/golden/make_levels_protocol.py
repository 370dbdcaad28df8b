"""Writes tests/golden/levels_protocol.json: for every case of tests/levels_protocol.py, the
collective sequence each rank of the row-sharded level build makes (the gloo rehearsal of
srt_levels_build), its outcome and each rank's own last level. Run from the repo root:

    python tests/golden/make_levels_protocol.py

tests/test_dist_gloo.py re-derives the sequences over gloo and compares them with this file;
tests/test_gpu_protocol.py compares the C library's collective logs (virtual ranks) with it."""
import json
import os
import socket
import sys

import torch.multiprocessing as mp

HERE = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, os.path.dirname(HERE))
sys.path.insert(0, os.path.dirname(os.path.dirname(HERE)))
import levels_protocol as lp  # noqa: E402


def _free_port():
    with socket.socket() as s:
        s.bind(("127.0.0.1", 0))
        return s.getsockname()[1]


def run_case(name):
    """[(rank, outcome, calls, row0, D, rel, own level)] of one case over gloo, rank order."""
    R = lp.CASES[name][1]
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=lp.gloo_worker, args=(r, R, port, name, q)) for r in range(R)]
    for p in procs:
        p.start()
    res = sorted([q.get(timeout=600) for _ in range(R)], key=lambda x: x[0])
    for p in procs:
        p.join(60)
        assert p.exitcode == 0
    return res


def main():
    out = {}
    for name in lp.CASES:
        res = run_case(name)
        seqs = {str([list(c) for c in x[2]]) for x in res}
        assert len(seqs) == 1, f"{name}: ranks differ"
        out[name] = {"R": lp.CASES[name][1], "outcome": res[0][1],
                     "calls": [list(c) for c in res[0][2]],
                     "own_levels": [int(x[6]) for x in res]}
        print(name, out[name]["outcome"], len(out[name]["calls"]), "calls", out[name]["own_levels"])
    with open(os.path.join(HERE, "levels_protocol.json"), "w") as f:
        json.dump(out, f, indent=1)


if __name__ == "__main__":
    main()
