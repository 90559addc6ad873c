"""The two segments of the r06_v10 ring-path miss scored by the batch paths (GPU box; diagnostic).

The failing session's evidence: the ring scorer gave 97.77742062925678 (stream 1, tick 164) and
99.25763811033005 (stream 0, tick 196); the ring read back at the end of that test and scored by
the linear batch scorer gave 98.04756931524389 and 99.22827564692939 against the oracle's
98.04756856169448 and 99.22792074878643.  Here the same segments, cut from the scenario's
signal (scripts/miss_r06.py), go through the linear float32 scorer and the fp64 path: if the
float32 scorer lands within ~1e-5 of the oracle on the true samples, the 3.5e-4 of the
read-back means the ring itself held other samples at the end of that run.
"""
import os
import sys

import numpy as np

ROOT = os.environ.get("GRAFT_REPO_ROOT", os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path.insert(0, ROOT)
sys.path.insert(0, os.path.join(ROOT, "tests"))
sys.path.insert(0, os.path.join(ROOT, "scripts"))


def main():
    import miss_r05
    import miss_r06
    from golden_io import matcher_fixture, template_arrays
    from easywakeword_amd import Engine
    fx, _ = matcher_fixture()
    tm, ts = template_arrays(fx)
    data = miss_r05.scenario()
    segs = []
    for st, tick, ln, rs, target, oracle in miss_r06.CASES:
        p = (tick - 1) // 16
        end = (16 * p + 16) * 1600
        j0 = end - 1 - ((end - 1 - rs) % 160000)
        if j0 + ln > end:
            j0 -= 160000
        segs.append(data[st][j0:j0 + ln].copy())
    print("scenario length", data.shape[1], "samples")
    e = Engine()
    e.set_template(tm, ts)
    for dt in ("float64", "float32"):
        _, _, s, _ = e.score(segs, candidate_dtype=dt)
        print(f"linear float32 scorer, candidate {dt}:", [repr(float(x)) for x in s])
    _, _, s64 = e.score_f64(segs)
    print("fp64 path:", [repr(float(x)) for x in s64])
    for (st, tick, ln, rs, target, oracle) in miss_r06.CASES:
        print(f"  stream {st} tick {tick}: oracle {oracle!r}, ring scorer {target!r}")
    e.close()


if __name__ == "__main__":
    main()
