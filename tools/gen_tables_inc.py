"""Turn the committed binary tables (tables/*.f64) into C initializer fragments (exact hex floats).

Used by the Makefile for both the HIP library and the oracle:
    python tools/gen_tables_inc.py <outdir>
writes <outdir>/cie_xyz.inc (471 rows x (x,y,z)), <outdir>/smits.inc (7 x 36) and
<outdir>/srgb_steps.inc (the 255 steps of the linear -> 8-bit map, tools/gen_srgb_steps.py).
"""
import struct
import sys
from pathlib import Path

ROOT = Path(__file__).resolve().parent.parent


def emit(src, dst, per_row):
    raw = (ROOT / "tables" / src).read_bytes()
    vals = struct.unpack("<%dd" % (len(raw) // 8), raw)
    rows = ["{" + ", ".join(v.hex() for v in vals[i:i + per_row]) + "}" for i in range(0, len(vals), per_row)]
    dst.write_text(",\n".join(rows) + "\n")


def main():
    out = Path(sys.argv[1])
    out.mkdir(parents=True, exist_ok=True)
    emit("cie1931_xyz_1nm_360_830.f64", out / "cie_xyz.inc", 3)
    emit("smits_basis_36bin.f64", out / "smits.inc", 36)
    emit("srgb_u8_steps.f64", out / "srgb_steps.inc", 255)


if __name__ == "__main__":
    main()
