"""Host-side checks of audio-ident_amd/csrc/aidfp_layout.h (compiled with g++, no GPU): K2's strip sizing
(peak_strip_len: every strip in one round when possible, never past kPeakStripMax, the bound of K2's 32-bit
buffer range), the hot-chunk bit order K1 and K2 share, and the CSR bucket key's bijection on the 26 bits a
landmark hash can set."""

import shutil
import subprocess
from pathlib import Path

import pytest

ROOT = Path(__file__).resolve().parent.parent
SRC = r"""
#include <cstdio>
#include <cstdlib>
#include <vector>
#include <set>
#define __host__
#define __device__
#include "aidfp_layout.h"
using namespace aid;
static int fails = 0;
#define CHECK(c) do { if (!(c)) { std::printf("FAIL %s:%d %s\n", __FILE__, __LINE__, #c); ++fails; } } while (0)
static int64_t count(const std::vector<int64_t> &f, int64_t L) { int64_t k = 0; for (auto x : f) k += (x + L - 1) / L; return k; }
int main() {
    // 256 x 10 s at 44.1 kHz (858 frames), 1024 slots: the smallest L that fits one round
    std::vector<int64_t> f(256, 858);
    int L = peak_strip_len(f.data(), (int)f.size(), 1024);
    CHECK(count(f, L) <= 1024 && count(f, L - 1) > 1024 && L >= kPeakStripMin);
    // a single 30-min clip spreads over the slots
    std::vector<int64_t> g(1, 155000);
    L = peak_strip_len(g.data(), 1, 1024);
    CHECK(count(g, L) <= 1024 && L < 200);
    // more long clips than slots: one strip per clip, but never past kPeakStripMax
    std::vector<int64_t> h(3000, 200000);
    L = peak_strip_len(h.data(), (int)h.size(), 1024);
    CHECK(L == kPeakStripMax);
    CHECK((int64_t)(kPeakStripMax + 2 * kPeakDT) * kBins * 4 < (int64_t)1 << 31);
    std::vector<int64_t> s(10, 5);
    CHECK(peak_strip_len(s.data(), (int)s.size(), 1024) == kPeakStripMin);
    // hot_bit: a bijection of the 64 chunks onto the 64 bits
    std::set<int> bits;
    for (int c = 0; c < 64; ++c) bits.insert(hot_bit(c));
    CHECK(bits.size() == 64 && *bits.begin() == 0 && *bits.rbegin() == 63);
    // bucket_key: injective on the 26 hash bits (k1: 31..22, k2: 21..12, dt: 5..0), < 2^26
    std::srand(7);
    std::set<uint32_t> keys;
    for (int i = 0; i < 200000; ++i) {
        const uint32_t k1 = std::rand() & 1023, k2 = std::rand() & 1023, dt = std::rand() & 63;
        const uint32_t h = (k1 << 22) | (k2 << 12) | dt;
        const uint32_t k = bucket_key(h);
        CHECK(k < (1u << 26));
        const uint32_t back = (((k >> 18) & 0xFF) << 22) | (((k >> 16) & 3) << 30) | (((k >> 9) & 0x7F) << 12) |
                              (((k >> 6) & 7) << 19) | (k & 0x3F);
        CHECK(back == h);
    }
    std::printf("%s\n", fails ? "FAILED" : "ok");
    return fails ? 1 : 0;
}
"""


@pytest.mark.skipif(shutil.which("g++") is None, reason="g++ not available")
def test_layout_header(tmp_path):
    src = tmp_path / "layout_check.cpp"
    src.write_text(SRC)
    exe = tmp_path / "layout_check"
    subprocess.run(["g++", "-std=c++17", "-O1", "-I", str(ROOT / "audio-ident_amd" / "csrc"), str(src), "-o", str(exe)],
                   check=True)
    out = subprocess.run([str(exe)], capture_output=True, text=True)
    assert out.returncode == 0 and out.stdout.strip().endswith("ok"), out.stdout
