"""Write the tag36h11 codebook include files from tools/tag36h11_gen.c output.

    gcc -O3 -march=native -fopenmp tools/tag36h11_gen.c -o /tmp/tag36h11_gen
    /tmp/tag36h11_gen > /tmp/tag36h11.txt          # ~30 min on 8 cores
    python tools/make_codebook.py /tmp/tag36h11.txt

Each input line is "id k code_rowmajor code_3x".  The same table goes to the
product (ros_vision_amd/csrc/at_tag36h11_codes.inc) and to the oracle
(oracle/ao_tag36h11_codes.inc); tests/test_family.py re-derives every entry's k.
"""
import sys
from pathlib import Path

ROOT = Path(__file__).resolve().parents[1]

HEADER = """/* tag36h11 code words (apriltag 3.x bit order) as {{id, code}} pairs.
 * Third-party data: cgpadwick/apriltag@3.3.0 tag36h11.c (587 codes), which the
 * reference fetches at build time (src/external/CMakeLists.txt:86-95) and uses
 * through tag36h11_create() (src/apriltags_cuda/src/apriltag_utils.cu:12) and
 * quad_decode_index (src/apriltags_cuda/src/apriltag_detect.cu:613).  It is not
 * vendored; this table is regenerated offline by tools/tag36h11_gen.c (the
 * AprilTag lexicode search: v0 = JavaRandom(361110).nextLong() mod 2^36, step
 * 982451653, minimum rotated Hamming distance 11, greedy rectangle complexity
 * >= 10) and written by tools/make_codebook.py.  Pinned by: ids 0..72 as
 * recalled from tag36h11.c (all 73 reproduced), and the codes of ids 554 and 585
 * read from the reference's fixture photographs test/data/colorimage.jpg and
 * grayimage.jpg (tools/read_fixture_codes.py), which the search emits at exactly
 * those ids (k = 6235272729 and 42477048845).  {n} entries. */
"""


def main(path):
    rows = []
    for line in Path(path).read_text().splitlines():
        parts = line.split()
        if len(parts) != 4:
            continue
        rows.append((int(parts[0]), int(parts[1]), int(parts[3], 16)))
    assert [r[0] for r in rows] == list(range(len(rows))), "ids must be 0..n-1"
    body = "".join("{%d, 0x%09xULL},\n" % (i, code) for i, _, code in rows)
    text = HEADER.format(n=len(rows)) + body
    for dst in (ROOT / "ros_vision_amd/csrc/at_tag36h11_codes.inc", ROOT / "oracle/ao_tag36h11_codes.inc"):
        dst.write_text(text)
        print("wrote", dst, len(rows), "entries")


if __name__ == "__main__":
    main(sys.argv[1])
