#!/usr/bin/env python3
"""Build libdls_hip.so variants with -D knobs for same-box A/B timing (tools/ab_bench.py).

    python tools/build_variants.py base: qU2:-DDLS_QUANT_U=2 noscalar:-DDLS_QUANT_SCALAR_SZ=0
"""
import concurrent.futures as cf
import os
import subprocess
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
CSRC = os.path.join(ROOT, "distributed_learning_simulator_amd", "csrc")
OUT = os.path.join(ROOT, "tools", "_variants")
SRCS = ["dls_runtime.hip", "fedavg.hip", "sign.hip", "quant.hip", "quant_fma.hip", "shapley.hip", "conv.hip",
        "infer.hip"]
FLAGS = ["--offload-arch=gfx950", "-O3", "-std=c++17", "-fPIC", "-ffp-contract=off"]


def build(name, defs, src=CSRC):
    d = os.path.join(OUT, name)
    os.makedirs(d, exist_ok=True)
    objs = []
    # DLS_VARIANT_SRCS=a.hip,b.hip: compile only those, link the in-tree build's
    # objects of the others (the knob does not touch them)
    only = [x for x in os.environ.get("DLS_VARIANT_SRCS", "").split(",") if x]
    for s in SRCS:
        if not os.path.exists(os.path.join(src, s)):  # a revision from before this source
            continue
        o = os.path.join(d, s.replace(".hip", ".o"))
        if only and s not in only:
            o = os.path.join(CSRC, "_build", s.replace(".hip", ".o"))
        else:
            subprocess.check_call(["hipcc", *FLAGS, *defs, "-I", src, "-c", os.path.join(src, s),
                                   "-o", o])
        objs.append(o)
    lib = os.path.join(OUT, f"libdls_{name}.so")
    subprocess.check_call(["hipcc", "--offload-arch=gfx950", "-shared", "-fPIC", "-o", lib, *objs])
    return lib


def main(specs):
    """spec = name:flag,flag[@git-rev]  (@rev builds the csrc of that git revision)"""
    jobs = []
    for spec in specs:
        spec, _, rev = spec.partition("@")
        name, _, flags = spec.partition(":")
        src = CSRC
        if rev:
            # <tree>/pkg/csrc + <tree>/include: dls_common.h's "../../include/dls_hip.h"
            # resolves to the revision's own header
            tree = os.path.join(OUT, f"_src_{rev}")
            src = os.path.join(tree, "pkg", "csrc")
            os.makedirs(src, exist_ok=True)
            os.makedirs(os.path.join(tree, "include"), exist_ok=True)
            for f in SRCS + ["dls_common.h", "quant_common.h"]:
                try:
                    blob = subprocess.check_output(
                        ["git", "-C", ROOT, "show",
                         f"{rev}:distributed_learning_simulator_amd/csrc/{f}"],
                        stderr=subprocess.DEVNULL)
                except subprocess.CalledProcessError:  # not in that revision
                    continue
                open(os.path.join(src, f), "wb").write(blob)
            blob = subprocess.check_output(["git", "-C", ROOT, "show", f"{rev}:include/dls_hip.h"])
            open(os.path.join(tree, "include", "dls_hip.h"), "wb").write(blob)
        jobs.append((name, [f for f in flags.split(",") if f], src))
    with cf.ThreadPoolExecutor(4) as ex:
        for lib in ex.map(lambda j: build(*j), jobs):
            print(lib)


if __name__ == "__main__":
    main(sys.argv[1:])
