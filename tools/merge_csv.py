#!/usr/bin/env python3
"""Concatenate rocprofv3 CSVs of one kind (same header) from several runs:
python tools/merge_csv.py <out.csv> <in1.csv> <in2.csv> ...  (inputs that
do not exist are skipped; the header is written once)."""
import os
import sys


def main():
    out, ins = sys.argv[1], sys.argv[2:]
    os.makedirs(os.path.dirname(out) or ".", exist_ok=True)
    header = None
    with open(out, "w") as fo:
        for p in ins:
            if not os.path.exists(p):
                continue
            with open(p) as fi:
                h = fi.readline()
                if header is None:
                    header = h
                    fo.write(h)
                for line in fi:
                    fo.write(line)


if __name__ == "__main__":
    main()
