#!/usr/bin/env python3
"""Diagnostic (NOT product build): the HIP library with hipcc's device
assembly passed through an assembly rewrite, assembled, linked and bundled by
hipcc's own steps (as tools/vgpr_banks.py --build-lib).
    python tools/diag/build_variant.py out.so <rewrite.py> [rewrite args ...]
The rewrite is run as `python rewrite.py in.s out.s [args]`.
"""
import os
import subprocess
import sys
import tempfile

ROOT = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))


def main():
    out_so, rewrite, rargs = os.path.abspath(sys.argv[1]), sys.argv[2], sys.argv[3:]
    src = os.path.join(ROOT, "subproc_amd", "csrc", "othello.hip")
    hipcc, llvm = "/opt/rocm/bin/hipcc", "/opt/rocm/lib/llvm/bin"
    inc = ["-I", os.path.join(ROOT, "include")]
    with tempfile.TemporaryDirectory() as tmp:
        j = lambda f: os.path.join(tmp, f)  # noqa: E731
        subprocess.check_call([hipcc, "--offload-arch=gfx950", "-O3", "-std=c++17", "-mllvm", "-pragma-unroll-threshold=200000", *inc,
                               "--cuda-device-only", "-S",
                               "-o", j("o.s"), src], stderr=subprocess.DEVNULL)
        subprocess.check_call([sys.executable, rewrite, j("o.s"), j("b.s"), *rargs])
        subprocess.check_call([os.path.join(llvm, "clang"), "-x", "assembler", "-target", "amdgcn-amd-amdhsa",
                               "-mcpu=gfx950", "-c", "-o", j("dev.o"), j("b.s")])
        subprocess.check_call([os.path.join(llvm, "ld.lld"), "-shared", "-o", j("o.hsaco"), j("dev.o")])
        subprocess.check_call([os.path.join(llvm, "clang-offload-bundler"), "-type=o", "-bundle-align=4096",
                               "-targets=host-x86_64-unknown-linux-gnu,hipv4-amdgcn-amd-amdhsa--gfx950",
                               "-input=/dev/null", "-input=" + j("o.hsaco"), "-output=" + j("o.hipfb")])
        subprocess.check_call([hipcc, "--offload-arch=gfx950", "-O3", "-std=c++17", "-fPIC", *inc, "--cuda-host-only",
                               "-Xclang", "-fcuda-include-gpubinary", "-Xclang", j("o.hipfb"), "-c", "-o", j("oth.o"),
                               src])
        subprocess.check_call([hipcc, "--offload-arch=gfx950", "-O3", "-std=c++17", "-fPIC", *inc, "-c",
                               "-o", j("td.o"), os.path.join(ROOT, "subproc_amd", "csrc", "td_table.hip")])
        subprocess.check_call([hipcc, "--offload-arch=gfx950", "-fPIC", "-shared",
                               "-Wl,--version-script=" + os.path.join(ROOT, "subproc_amd", "csrc", "exports.map"),
                               "-o", out_so, j("oth.o"), j("td.o")])


if __name__ == "__main__":
    main()
