"""Does a built library's gfx950 code object hold a kernel symbol?  HIP
aborts the process -- in the launch and in hipFuncGetAttributes alike
(tools/dbg/missing_symbol_probe.hip, profiles/r06/missing_symbol_probe.txt)
-- when a host stub's device code is missing, so the check has to read the
code objects before the library is loaded: llvm-objdump --offloading
extracts them, llvm-readelf lists their symbols."""
import glob
import os
import shutil
import subprocess
import tempfile

LLVM = "/opt/rocm/lib/llvm/bin"


def device_symbols(lib: str) -> set:
    tmp = tempfile.mkdtemp()
    try:
        shutil.copy(lib, os.path.join(tmp, "lib.so"))
        subprocess.run([f"{LLVM}/llvm-objdump", "--offloading", "lib.so"], cwd=tmp, check=True,
                       capture_output=True)
        syms = set()
        for co in glob.glob(os.path.join(tmp, "lib.so.*gfx950*")):
            out = subprocess.run([f"{LLVM}/llvm-readelf", "--symbols", co], check=True,
                                 capture_output=True, text=True).stdout
            syms.update(line.split()[-1] for line in out.splitlines() if "FUNC" in line)
        return syms
    finally:
        shutil.rmtree(tmp, ignore_errors=True)


def narrow_symbol(unr: int, hu: int, ga: int, gv: int) -> str:
    return (f"_ZN3mmb23utt_narrow_fused_kernelILi{unr}ELi{hu}ELi{ga}ELi{gv}ELb0EEEv"
            "NS_15NarrowFusedArgsE")
