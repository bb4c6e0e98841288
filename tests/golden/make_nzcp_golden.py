"""Writes tests/golden/nzcp_cases.json: the nzcp witness parity cases
(tests/nzcp_cases.py) with the records of the CPU restatement
(oracle/nzcp_circuit.py). The restatement itself is pinned by the reference's own
KATs in tests/test_nzcp_oracle.py; this file freezes its outputs so a change to
either side shows up as a diff.

    python tests/golden/make_nzcp_golden.py
"""
import json
import os
import sys

HERE = os.path.dirname(os.path.abspath(__file__))
sys.path[:0] = [os.path.dirname(os.path.dirname(HERE)), os.path.dirname(HERE)]

import nzcp_cases  # noqa: E402


def main():
    cases = nzcp_cases.all_cases()
    out = {"generator": "tests/golden/make_nzcp_golden.py", "cases": cases,
           "expected": [nzcp_cases.oracle_record(c) for c in cases]}
    with open(os.path.join(HERE, "nzcp_cases.json"), "w") as f:
        json.dump(out, f, indent=0, sort_keys=True)
        f.write("\n")
    print(f"{len(cases)} cases")


if __name__ == "__main__":
    main()
