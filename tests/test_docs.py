"""The documents cite files that exist.

DESIGN.md, BASELINE.md, INTEGRATION.md and README.md point the reader at
evidence (`profiles/...`), tools, tests and sources by repository path. A
path that was renamed or never committed leaves a claim without its
evidence, so every backticked repository path in them must match at least
one file (`*` patterns allowed). CPU only.
"""
import glob
import os
import re

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
DOCS = ["DESIGN.md", "BASELINE.md", "INTEGRATION.md", "README.md"]
TOP = ("profiles/", "tools/", "tests/", "tulips_amd/", "include/", "oracle/",
       "benchlib/", "integration/")
# built or generated at run time, never committed
BUILT = ("oracle/_ref", "tulips_amd/libtulips_csum.so", "benchlib/libtulips_csum_bench.so",
         "tests/native/runtime_check", "gpurun_out/")
# the reference tree's own paths, cited as `file:line` of /root/reference
# (its public headers and tests), or as where an integrator puts a file there
REFERENCE = ("include/tulips", "tests/stack/")


# a bare evidence file name (`bench_r06aw.json`, `rocprof_r06aw_*`) is one
# under profiles/
EVIDENCE = re.compile(r"^[a-z][a-z0-9_]*_r\d\d[a-z]*[A-Za-z0-9_*.-]*$")


def cited_paths(text):
    for tok in re.findall(r"`([^`\s]+)`", text):
        path = tok.split(":")[0].split("::")[0].rstrip(".,;")
        if path.startswith(TOP) and not path.startswith(BUILT + REFERENCE):
            yield path
        elif "/" not in path and EVIDENCE.match(path):
            yield "profiles/" + path


@pytest.mark.parametrize("doc", DOCS)
def test_cited_repository_paths_exist(doc):
    with open(os.path.join(ROOT, doc)) as f:
        text = f.read()
    missing = sorted({p for p in cited_paths(text)
                      if not glob.glob(os.path.join(ROOT, p.rstrip("/")))})
    assert not missing, f"{doc} cites paths that do not exist: {missing}"
