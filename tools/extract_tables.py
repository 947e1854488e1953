"""Extract the spectral data tables the hot path reads into raw little-endian f64 files.

Data only: the CIE 1931 2-degree colour-matching functions at 1 nm (360..830 nm, 471 rows) and the
seven Smits (1999) 36-bin basis spectra, as tabulated in the reference's
`raytracer/src/color.rs:286-1982`. This script is run once in the build container (where
/root/reference exists); its outputs under tables/ are committed so that nothing reads the
reference at run time.

    python tools/extract_tables.py [/root/reference/raytracer/src/color.rs]
"""
import re
import struct
import sys
from pathlib import Path

SRC = Path(sys.argv[1] if len(sys.argv) > 1 else "/root/reference/raytracer/src/color.rs")
OUT = Path(__file__).resolve().parent.parent / "tables"

NUM = re.compile(r"^\s*(-?[0-9][0-9_]*\.?[0-9_]*(?:e-?[0-9]+)?),\s*$")


def block(lines, header):
    start = next(i for i, l in enumerate(lines) if l.startswith(header))
    vals = []
    for l in lines[start + 1:]:
        if l.strip().startswith("]"):
            break
        m = NUM.match(l)
        if m:
            vals.append(float(m.group(1).replace("_", "")))
    return vals


def main():
    lines = SRC.read_text().splitlines()
    cie = [block(lines, f"pub const CIE_{c}: [f64; 471]") for c in "XYZ"]
    assert all(len(c) == 471 for c in cie), [len(c) for c in cie]
    names = ["WHITE", "CYAN", "MAGENTA", "YELLOW", "RED", "GREEN", "BLUE"]
    smits = [block(lines, f"static {n}_SPECTRUM: Spectrum") for n in names]
    assert all(len(s) == 36 for s in smits), [len(s) for s in smits]
    OUT.mkdir(exist_ok=True)
    # row-major [471][3] (x, y, z per nm) and [7][36]
    with open(OUT / "cie1931_xyz_1nm_360_830.f64", "wb") as f:
        for i in range(471):
            f.write(struct.pack("<3d", cie[0][i], cie[1][i], cie[2][i]))
    with open(OUT / "smits_basis_36bin.f64", "wb") as f:
        for s in smits:
            f.write(struct.pack("<36d", *s))
    print("CIE_Y sum", sum(cie[1]))


if __name__ == "__main__":
    main()
