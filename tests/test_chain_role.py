"""Host check of chain_kernel's dispatch-slot -> role permutation (gpk_internal.h chain_role):
every slot of a factor's grid row maps to exactly one role (T*TC tiles + the pivot chain), for
both rows, over a range of tile counts with and without augmented columns.  A role missing from
the grid would leave the persistent inverse waiting forever, so this is checked without a GPU.

The function is compiled as plain C++ from the header text (it is __host__ __device__ and uses
no HIP API)."""
import os
import re
import shutil
import subprocess

import pytest

HDR = os.path.join(os.path.dirname(__file__), "..", "gaussian-process-slover-for-high-freq-pde_amd",
                   "csrc", "gpk_internal.h")

MAIN = r"""
#include <cstdio>
#include <vector>
int main() {
  int bad = 0;
  for (int T = 1; T <= 24; ++T)
    for (int extra = 0; extra <= 48; extra += T) {
      const int TC = T + extra, nt = T * TC;
      for (int m = 0; m < 2; ++m) {
        std::vector<int> seen(nt + 1, 0);
        for (int x = 0; x <= nt; ++x) {
          const int r = chain_role(m, x, T, TC);
          if (r < 0 || r > nt) { ++bad; continue; }
          ++seen[r];
        }
        for (int r = 0; r <= nt; ++r) bad += seen[r] != 1;
      }
    }
  // C4 (T = 8, TC = 24): the chain is the last slot of row 0 and the first of row 1
  bad += chain_role(0, 192, 8, 24) != 192;
  bad += chain_role(1, 0, 8, 24) != 192;
  std::printf("%d\n", bad);
  return 0;
}
"""


@pytest.mark.skipif(shutil.which("g++") is None, reason="needs g++")
def test_chain_role_is_a_bijection(tmp_path):
    src = open(HDR).read()
    m = re.search(r"__host__ __device__ inline int chain_role\(.*?\n}\n", src, re.S)
    assert m, "chain_role not found in gpk_internal.h"
    fn = m.group(0).replace("__host__ __device__ ", "")
    cpp = tmp_path / "role.cpp"
    cpp.write_text(fn + MAIN)
    exe = tmp_path / "role"
    subprocess.run(["g++", "-O1", "-std=c++17", str(cpp), "-o", str(exe)], check=True)
    out = subprocess.run([str(exe)], check=True, capture_output=True, text=True).stdout.strip()
    assert out == "0"


SPD = os.path.join(os.path.dirname(HDR), "spdinv.hip")

MULTI_MAIN = r"""
#include <cstdio>
#include <vector>
#include <algorithm>
int main() {
  int bad = 0;
  for (int T = 1; T <= 80; ++T) {
    const int MT = (T + 1) / 2, nwg = 1 + MT * (MT - 1) / 2;
    std::vector<int> own(T * T, 0);
    for (int g = 0; g < nwg; ++g) {
      int R, c0, dm, n = 0;
      multi_role(g, R, c0, dm);
      for (int s = 0; s < 7; ++s) {
        if (s < 4 && c0 < 0) continue;
        if (s >= 4 && !((dm >> (s - 4)) & 1)) continue;
        int I, J;
        multi_slot(s, R, c0, I, J);
        if (I >= T || J > I) continue;
        ++own[I * T + J];
        ++n;
      }
      if (R >= 3 && n > 5) ++bad;   // no workgroup past macro row 2 updates more than 5 tiles
      if (R == 2 && n > 6) ++bad;
    }
    for (int I = 0; I < T; ++I)
      for (int J = 0; J < T; ++J) bad += own[I * T + J] != (J <= I ? 1 : 0);
  }
  std::printf("%d\n", bad);
  return 0;
}
"""


@pytest.mark.skipif(shutil.which("g++") is None, reason="needs g++")
def test_multi_role_covers_lower_triangle(tmp_path):
    """chain_multi_kernel's workgroup -> tiles map (spdinv.hip multi_role / multi_slot): every
    lower tile of a T x T factor has exactly one owner, and the diagonal block's tiles are spread
    so that no workgroup from macro row 3 on holds more than five tiles."""
    src = open(SPD).read()
    fns = []
    for name in ("multi_slot", "multi_role"):
        m = re.search(r"__host__ __device__ inline void " + name + r"\(.*?\n}\n", src, re.S)
        assert m, name + " not found in spdinv.hip"
        fns.append(m.group(0).replace("__host__ __device__ ", ""))
    cpp = tmp_path / "multi.cpp"
    cpp.write_text("\n".join(fns) + MULTI_MAIN)
    exe = tmp_path / "multi"
    subprocess.run(["g++", "-O1", "-std=c++17", str(cpp), "-o", str(exe)], check=True)
    out = subprocess.run([str(exe)], check=True, capture_output=True, text=True).stdout.strip()
    assert out == "0"
