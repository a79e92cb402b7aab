"""Source stamp of the ring GraphSum: a sha256 over the files that decide what the kernel does
(kernel, schedule builder, LDS-DMA helpers, fused epilogues).  tools/traffic.py writes it into
profiles/traffic_graphsum.json next to the PMC bytes; bench.py reports those bytes as
`roofline.traffic` only while the stamp still matches the sources it runs (else null).
"""
import hashlib
import os
import re

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
GRAPHSUM_SOURCES = (
    "parallel-gcn_amd/csrc/k_graphsum_ring.hip",
    "parallel-gcn_amd/csrc/host/ring.cpp",
    "parallel-gcn_amd/csrc/lds_dma.hpp",
    "parallel-gcn_amd/csrc/gs_epilogue.hpp",
)


def code_only(text):
    """The source without its comments and blank space (a comment edit keeps the stamp)."""
    text = re.sub(r"/\*.*?\*/", " ", text, flags=re.S)
    text = re.sub(r"//[^\n]*", " ", text)
    return " ".join(text.split())


def graphsum_stamp(root=REPO):
    h = hashlib.sha256()
    for rel in GRAPHSUM_SOURCES:
        h.update(rel.encode())
        with open(os.path.join(root, rel), encoding="utf-8") as f:
            h.update(code_only(f.read()).encode())
    return h.hexdigest()[:16]


if __name__ == "__main__":
    print(graphsum_stamp())
