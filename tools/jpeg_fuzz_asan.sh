#!/bin/bash
# Host-only AddressSanitizer run of the JPEG marker parser + entropy decoder (mx_jpeg.cpp) over
# mutated PIL-encoded files: random byte flips in the headers and the scan, truncations and
# over-subscribed Huffman counts. CPU only (no GPU code involved). Usage: tools/jpeg_fuzz_asan.sh [N]
set -e
cd "$(dirname "$0")/.."
out=/tmp/mx_jpeg_fuzz
mkdir -p $out
cat > $out/drv.cpp <<'CPP'
#include <stdio.h>
#include <stdlib.h>
#include <stdarg.h>
#include <vector>
#include "mx_det.h"
namespace mx { void set_error(const char* fmt, ...) { (void)fmt; } }
int main(int argc, char** argv) {
  int bad = 0, ok = 0;
  for (int a = 1; a < argc; ++a) {
    FILE* f = fopen(argv[a], "rb");
    std::vector<uint8_t> d;
    int c;
    while ((c = fgetc(f)) != EOF) d.push_back((uint8_t)c);
    fclose(f);
    mx_jpeg_info info;
    if (mx_jpeg_parse(d.data(), (int64_t)d.size(), &info) != 0) { ++bad; continue; }
    std::vector<int16_t> coefs((size_t)info.coef_total);
    if (mx_jpeg_decode_coefs(d.data(), (int64_t)d.size(), &info, coefs.data()) != 0) ++bad; else ++ok;
  }
  printf("decoded %d rejected %d\n", ok, bad);
  return 0;
}
CPP
g++ -O1 -g -fsanitize=address,undefined -fno-omit-frame-pointer -std=c++17 -Iinclude \
    -D__HIP_PLATFORM_AMD__ -I/opt/rocm/include \
    robust-object-detection_amd/csrc/mx_jpeg.cpp $out/drv.cpp -o $out/drv
python3 - "$out" "${1:-400}" <<'PY'
import io, sys, random
import numpy as np
from PIL import Image
out, n = sys.argv[1], int(sys.argv[2])
rng = random.Random(0)
for i in range(n):
    a = np.random.default_rng(i).integers(0, 255, (rng.randint(8, 80), rng.randint(8, 80), 3), dtype=np.uint8)
    b = io.BytesIO()
    Image.fromarray(a).save(b, format="JPEG", quality=rng.choice([50, 90, 95]), subsampling=rng.choice([0, 1, 2]))
    d = bytearray(b.getvalue())
    kind = i % 4
    if kind == 0:    # header byte flips
        for _ in range(rng.randint(1, 6)):
            d[rng.randrange(2, min(len(d), 700))] = rng.randrange(256)
    elif kind == 1:  # scan byte flips
        for _ in range(rng.randint(1, 20)):
            d[rng.randrange(len(d) // 2, len(d))] = rng.randrange(256)
    elif kind == 2:  # truncation
        d = d[:rng.randrange(4, len(d))]
    else:            # Huffman counts inflated
        j = d.find(b"\xff\xc4")
        if j > 0:
            d[j + 5 + rng.randrange(16)] = rng.randrange(256)
    open(f"{out}/f{i:04d}.jpg", "wb").write(d)
PY
ASAN_OPTIONS=detect_leaks=0 $out/drv $out/f*.jpg
