// Host build of csrc/f29.h (NZ_HD = inline without HIP): reads test vectors on stdin and
// prints the library's results, which tests/test_f29_host.py compares with exact integers.
//   op 1: mul_shoup(x, w, ws)      op 2: mul_shoup_x2 (both results)
//   op 3: mul_lo261(a, b)          op 4: mul29<Fr29>(a, b)
//   op 5: fr_to261(Fr, 8 words)    op 6: fr_from261(F29) (8 words out)
// Input lines: "<op> <hex limbs of each operand, 9 per F29>"; output: 9 hex limbs per result.
#include <cstdio>
#include <cstdlib>
#include <cstring>

#include "../../nzcb-circom_amd/csrc/f29.h"

using namespace nzcb;

static bool rd(F29& x) {
  for (int i = 0; i < 9; i++)
    if (std::scanf("%x", &x.v[i]) != 1) return false;
  return true;
}
static void wr(const F29& x) {
  for (int i = 0; i < 9; i++) std::printf("%x%c", x.v[i], i == 8 ? '\n' : ' ');
}

int main() {
  int op;
  while (std::scanf("%d", &op) == 1) {
    F29 a, b, c, d, e, f;
    if (op == 1) {
      rd(a); rd(b); rd(c);
      wr(mul_shoup(a, b, c));
    } else if (op == 2) {
      rd(a); rd(b); rd(c); rd(d); rd(e); rd(f);
      F29 r1, r2;
      mul_shoup_x2(a, b, c, d, e, f, r1, r2);
      wr(r1);
      wr(r2);
    } else if (op == 3) {
      rd(a); rd(b);
      wr(mul_lo261(a, b));
    } else if (op == 4) {
      rd(a); rd(b);
      wr(mul29<Fr29>(a, b));
    } else if (op == 5) {
      Fr x;
      for (int i = 0; i < 8; i++) std::scanf("%x", &x.v[i]);
      wr(fr_to261(x));
    } else if (op == 6) {
      rd(a);
      const Fr y = fr_from261(a);
      for (int i = 0; i < 8; i++) std::printf("%x%c", y.v[i], i == 7 ? '\n' : ' ');
    } else {
      return 2;
    }
  }
  return 0;
}
