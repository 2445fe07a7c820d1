"""Loaders for the committed fixtures in tests/golden/ (made by
tests/golden/make_golden.py from the reference's own compiled sources)."""
import json
import os

import numpy as np

GOLDEN = os.path.join(os.path.dirname(os.path.abspath(__file__)), "golden")


def kat():
    with open(os.path.join(GOLDEN, "kat.json")) as f:
        return json.load(f)["cases"]


def kat_data(case, oracle=None):
    if "data" in case:
        return bytes.fromhex(case["data"])
    seed, length = case["data_splitmix"]
    return oracle.splitmix_bytes(length, seed=seed).tobytes()


def adversarial():
    with np.load(os.path.join(GOLDEN, "adversarial.npz"), allow_pickle=False) as z:
        return {k: z[k] for k in z.files}


def digests():
    with open(os.path.join(GOLDEN, "digests.json")) as f:
        return json.load(f)


# expected-array name -> (arena kind, mode, use seeds)
ADV_CASES = {
    "raw_noseed": ("arena", 0, False),
    "raw_seed": ("arena", 0, True),
    "inet_seed": ("arena", 1, True),
    "tcp": ("arena", 2, False),
    "tcp_complement": ("arena", 0x102, False),
    "zeros_raw_seed": ("zeros", 0, True),
    "zeros_inet_noseed": ("zeros", 1, False),
    "ones_raw_seed": ("ones", 0, True),
    "ones_tcp": ("ones", 2, False),
}


def adv_arena(adv, kind):
    a = adv["arena"]
    if kind == "zeros":
        return np.zeros_like(a)
    if kind == "ones":
        return np.full_like(a, 0xFF)
    return a
