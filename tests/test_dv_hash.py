"""dv_hash_words (the probe's word-at-a-time dvUniqueId hash, dk_uri.h) equals dv_emit + HashSink
(the byte stream the commit tail's keys are hashed from) for every alignment and length of
pathOrInlineDv, with and without an offset, and refuses non-ASCII input (dv_emit validates it).
Built on the host with g++ from the shared header (DeletionVectorDescriptor.java:167-174)."""
import os
import subprocess

import pytest

HERE = os.path.dirname(os.path.abspath(__file__))
CSRC = os.path.join(HERE, "..", "delta_amd", "csrc")

PROG = r'''
#include <cstdio>
#include <cstring>
#include <cstdlib>
#include "dk_uri.h"
using namespace dk;
static uint64_t ref(const uint8_t* st, int stn, const uint8_t* pid, int pidn, bool ho, int off, uint32_t seed, int* rc) {
  HashSink k; k.hs.init(kHashSeed(seed)); k.n = 0;
  *rc = dv_emit(true, st, stn, pid, pidn, ho, off, k);
  return k.hs.final_(k.n);
}
int main() {
  static uint8_t buf[4096 + 64];
  uint32_t x = 12345;
  auto rnd = [&]() { x = x * 1103515245u + 12345u; return (x >> 8); };
  int checked = 0, refused = 0;
  for (int it = 0; it < 200000; it++) {
    memset(buf, 0xAB, sizeof buf);
    const int align = rnd() % 8, pidn = rnd() % 70, stn = rnd() % 3;
    uint8_t* st = buf + 8; uint8_t* pid = buf + 32 + align;
    const bool nonascii = rnd() % 50 == 0;
    for (int i = 0; i < stn; i++) st[i] = "uip"[rnd() % 3];
    for (int i = 0; i < pidn; i++) pid[i] = 33 + rnd() % 90;
    if (nonascii && pidn) pid[rnd() % pidn] = 0xC3;
    const bool ho = rnd() % 2; const int off = ho ? (int)(rnd() % 2000000) - 1000 : 0;
    const uint32_t seed = rnd() % 3;
    uint64_t got = 0;
    const bool ok = dv_hash_words(st, stn, pid, pidn, ho, off, seed, &got);
    int rc = 0;
    const uint64_t want = ref(st, stn, pid, pidn, ho, off, seed, &rc);
    if (!ok) { refused++; if (!nonascii) { printf("refused ASCII input at %d\n", it); return 1; } continue; }
    if (rc != 0 || got != want) { printf("mismatch at %d: pidn %d align %d\n", it, pidn, align); return 1; }
    checked++;
  }
  printf("ok %d %d\n", checked, refused);
  return 0;
}
'''


def test_dv_hash_words_matches_dv_emit(tmp_path):
    src = tmp_path / "dvh.cpp"
    src.write_text(PROG)
    exe = tmp_path / "dvh"
    subprocess.run(["g++", "-O2", "-std=c++17", "-I", CSRC, str(src), "-o", str(exe)], check=True)
    out = subprocess.run([str(exe)], capture_output=True, text=True)
    assert out.returncode == 0, out.stdout + out.stderr
    assert out.stdout.startswith("ok "), out.stdout
    checked, refused = map(int, out.stdout.split()[1:3])
    assert checked > 150000 and refused > 0
