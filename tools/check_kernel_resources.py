"""Build-time check of kernel register / scratch budgets whose correctness or residency depends on them (Makefile).

res_proj_kernel: its ring waits (rp_wait_case) count this wave's vector-memory operations by hand; a compiler spill to
scratch would add loads / stores the count does not know about, and it must stay <= 104 VGPRs to co-reside with the
other sampler stream's gate GEMM (res_proj.hip). gate_ws_kernel: its first waves' vmcnt waits count the ring DMAs by
hand (no scratch allowed either) and two waves per SIMD need <= 256 registers.
Usage: check_kernel_resources.py REMARKS_FILE KERNEL_SUBSTRING MAX_VGPRS"""
import re
import sys


def main():
    path, name, max_vgpr = sys.argv[1], sys.argv[2], int(sys.argv[3])
    text = open(path).read()
    blocks = re.split(r"remark: Function Name: ", text)[1:]
    seen = 0
    bad = []
    for b in blocks:
        fn = b.split()[0]
        if name not in fn:
            continue
        seen += 1
        get = lambda k: int(re.search(k + r": (\d+)", b).group(1))
        vgpr, agpr = get("VGPRs"), get("AGPRs")
        scratch = get("ScratchSize \\[bytes/lane\\]")
        spill = get("VGPRs Spill") + get("SGPRs Spill")
        if vgpr + agpr > max_vgpr or scratch or spill:
            bad.append(f"{fn}: {vgpr} VGPRs + {agpr} AGPRs (max {max_vgpr}), scratch {scratch} B/lane, spills {spill}")
    if not seen:
        sys.exit(f"check_kernel_resources: no kernel matching {name!r} in {path}")
    if bad:
        sys.exit("check_kernel_resources: " + "; ".join(bad))
    print(f"check_kernel_resources: {seen} {name} instance(s) within {max_vgpr} registers, no scratch")


if __name__ == "__main__":
    main()
