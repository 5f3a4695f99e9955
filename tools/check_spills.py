"""Compile the hot HIP kernels with --save-temps and list every kernel that uses
scratch (register spills): a spill in a main loop turns into vector-memory
traffic and extra vmcnt waits (a 3x weight-gradient slowdown went in unnoticed
once). Run after touching a kernel:

    python tools/check_spills.py [gemm flash_attn_d64 ...]
"""
import os
import re
import subprocess
import sys
import tempfile

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
# kernels known to spill a few bytes outside their main loop (setup / epilogue reloads)
KNOWN = {"gemm_sk_kernel": 64, "gemm_kernelILi256ELi320ELb0ELb0ELi1": 128, "bwd_dq_kernelILi2": 32}


def main():
    names = sys.argv[1:] or ["gemm", "flash_attn_d64", "decode_gemm", "paged_decode_mfma", "conv"]
    bad = 0
    with tempfile.TemporaryDirectory() as d:
        for n in names:
            src = os.path.join(ROOT, "csrc", "kernels", n + ".hip")
            subprocess.run(["/opt/rocm/bin/hipcc", "--offload-arch=gfx950", "-O3", "-std=c++17",
                            "-I", os.path.join(ROOT, "csrc", "kernels"), "-c", src, "-o",
                            os.path.join(d, n + ".o"), "--save-temps"], cwd=d, check=True,
                           stdout=subprocess.DEVNULL, stderr=subprocess.DEVNULL)
            asm = open(os.path.join(d, f"{n}-hip-amdgcn-amd-amdhsa-gfx950.s")).read()
            for k in re.findall(r"^\s*\.amdhsa_kernel (\S+)$", asm, re.M):
                i = asm.index(".amdhsa_kernel " + k)
                seg = asm[i: asm.find(".end_amdhsa_kernel", i)]
                scratch = int(re.search(r"\.amdhsa_private_segment_fixed_size (\d+)", seg).group(1))
                if scratch:
                    allowed = max([v for key, v in KNOWN.items() if key in k] or [0])
                    flag = "ok (known)" if scratch <= allowed else "SPILL"
                    bad += flag == "SPILL"
                    print(f"{n}: {k[:90]} scratch {scratch} B  {flag}")
    sys.exit(1 if bad else 0)


if __name__ == "__main__":
    main()
