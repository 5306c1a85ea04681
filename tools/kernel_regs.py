"""Register / spill / LDS counts of the gfx950 kernels in a built object (code-object metadata).

    python3 tools/kernel_regs.py [build/obj/tcpcsum_kernels.o] [name-substring ...]

Extracts the .hip_fatbin section, unbundles the gfx950 code object and prints one
line per kernel: VGPRs, AGPRs, VGPR / SGPR spills, scratch bytes per lane, name.
Also `--isa <substring>`: the disassembly of the matching kernels' store
instructions (checks the cache-policy bits of the write-through stores).
"""
import os
import re
import subprocess
import sys
import tempfile

LLVM = "/opt/rocm/lib/llvm/bin"


def code_object(obj: str, tmp: str) -> str:
    fat = os.path.join(tmp, "fat.bin")
    subprocess.run([f"{LLVM}/llvm-objcopy", "--dump-section", f".hip_fatbin={fat}", obj, os.path.join(tmp, "x.o")],
                   check=True)
    co = os.path.join(tmp, "k.co")
    subprocess.run([f"{LLVM}/clang-offload-bundler", "--type=o", "--unbundle", f"--input={fat}",
                    "--targets=hipv4-amdgcn-amd-amdhsa--gfx950", f"--output={co}"], check=True)
    return co


def kernels(co: str):
    notes = subprocess.run([f"{LLVM}/llvm-readelf", "--notes", co], capture_output=True, text=True, check=True).stdout
    for b in notes.split("  - .agpr_count")[1:]:
        g = lambda k: (re.search(rf"\.{k}:\s+(\S+)", b) or [None, "?"])[1]  # noqa: E731
        yield dict(name=g("name"), vgpr=g("vgpr_count"), agpr=b.split()[1] if b.split() else "?",
                   vspill=g("vgpr_spill_count"), sspill=g("sgpr_spill_count"), scratch=g("private_segment_fixed_size"))


def main():
    args = sys.argv[1:]
    isa = None
    if "--isa" in args:
        i = args.index("--isa")
        isa = args[i + 1]
        del args[i:i + 2]
    obj = args[0] if args and args[0].endswith(".o") else "build/obj/tcpcsum_kernels.o"
    subs = [a for a in args if not a.endswith(".o")]
    with tempfile.TemporaryDirectory() as tmp:
        co = code_object(obj, tmp)
        for k in kernels(co):
            if subs and not any(s in k["name"] for s in subs):
                continue
            print(f"vgpr {k['vgpr']:>4} agpr {k['agpr']:>3} vspill {k['vspill']:>3} sspill {k['sspill']:>3} "
                  f"scratch {k['scratch']:>4}  {k['name']}")
        if isa:
            dis = subprocess.run([f"{LLVM}/llvm-objdump", "-d", "--no-show-raw-insn", co], capture_output=True,
                                 text=True, check=True).stdout
            cur = None
            for line in dis.splitlines():
                m = re.match(r"^[0-9a-f]+ <(.*)>:", line)
                if m:
                    cur = m.group(1)
                    continue
                if cur and isa in cur and "store" in line:
                    print(f"{cur[:60]}: {line.strip()}")


if __name__ == "__main__":
    main()
