"""Regenerate the parity fixtures in tests/golden/ from the CPU oracle.

    python tests/golden/make_golden.py

Each fixture = the full apd_problem of one seeded synthetic case (tests/cases.py; priors of the
REFINE_* case come from an oracle FIRST_INIT pass over the neighbouring views) + the oracle's outputs.
The reference itself cannot run in this pipeline, so these vectors pin the oracle and
the HIP path to each other and to themselves over time ("parity unpinned" against the reference).
"""
import os
import sys

HERE = os.path.dirname(os.path.abspath(__file__))
sys.path[:0] = [os.path.dirname(HERE), os.path.join(os.path.dirname(os.path.dirname(HERE)), "apde-mvs_amd")]

import cases  # noqa: E402
import golden_io  # noqa: E402
import oracle_lib  # noqa: E402

FIXTURES = ("first_n4", "refine_iter_apd_geom_sa")


def main():
    lib = oracle_lib.load()
    orun = lambda arr: oracle_lib.run(lib, arr)
    for name in FIXTURES:
        arr = cases.make_case(name, orun)
        out = oracle_lib.run(lib, arr)
        path = os.path.join(HERE, name + ".npz")
        golden_io.save(path, arr, out)
        print(f"{path}: {os.path.getsize(path)} bytes, weak_count={int(out.weak_count[0])}")


if __name__ == "__main__":
    main()
