// lazy_check.hip -- host run of csrc/lazy.hpp (the accumulate's redundant
// Fq form) for tests/test_lazy_field.py, which checks every line with Python
// integers:
//   lazy_check POINTS N_POINTS SEED
// POINTS: binary affine G1 points (x, y as 12 little-endian u32 each, device
// Montgomery form).  Output lines (hex limbs, most significant last):
//   mul|sqr|mulsub|canon|zero <operands...> <result>
//   acc <step> <X> <Y> <ZZ> <ZZZ>   canonical XYZZ after each madd
#include <cstdio>
#include <cstdlib>
#include <vector>

#include "../zero-knowledge-proofs_amd/csrc/lazy.hpp"

using namespace zk;

static uint64_t g_s;
static uint64_t rnd() {
  uint64_t x = (g_s += 0x9e3779b97f4a7c15ull);
  x = (x ^ (x >> 30)) * 0xbf58476d1ce4e5b9ull;
  x = (x ^ (x >> 27)) * 0x94d049bb133111ebull;
  return x ^ (x >> 31);
}
static Fq rnd_fq() {   // uniform in [0, p)
  for (;;) {
    Fq a;
    for (int i = 0; i < 12; i++) a.v[i] = (uint32_t)rnd();
    a.v[11] &= 0x1fffffffu;
    bool lt = false;
    for (int i = 11; i >= 0; i--)
      if (a.v[i] != FqParams::MOD[i]) {
        lt = a.v[i] < FqParams::MOD[i];
        break;
      }
    if (lt) return a;
  }
}
// operand shapes the accumulate produces: canonical, negated, a sum of two
// (limbs < 2^29), a difference of two, a product output
static Fl rnd_fl(int shape) {
  const Fl a = fl_from_fq(rnd_fq()), b = fl_from_fq(rnd_fq());
  switch (shape) {
    case 0: return a;
    case 1: return fl_neg(a);
    case 2: return fl_add(a, b);
    case 3: return fl_sub(a, b);
    default: return fl_mul(a, b);
  }
}
static void put(const Fl& a) {
  printf(" ");
  for (int i = 0; i < FL_N; i++) printf("%s%x", i ? "," : "", (uint32_t)a.v[i]);
}
static void put(const Fq& a) {
  printf(" ");
  for (int i = 0; i < 12; i++) printf("%s%x", i ? "," : "", a.v[i]);
}

int main(int argc, char** argv) {
  if (argc < 4) return 2;
  const int np = atoi(argv[2]);
  g_s = strtoull(argv[3], nullptr, 0);
  std::vector<Fq> pts(2 * (size_t)np);
  FILE* f = fopen(argv[1], "rb");
  if (!f || fread(pts.data(), sizeof(Fq), pts.size(), f) != pts.size()) return 3;
  fclose(f);
  for (int t = 0; t < 400; t++) {
    const Fl a = rnd_fl(t % 5), b = rnd_fl((t / 5) % 5);
    printf("mul");
    put(a); put(b); put(fl_mul(a, b));
    printf("\nsqr");
    put(a); put(fl_sqr(a));
    static const int cshape[4] = {0, 1, 3, 4};
    const Fl c = rnd_fl(cshape[(t / 25) % 4]), d = rnd_fl(t % 4 == 2 ? 0 : t % 4);
    const Fl e = rnd_fl(t % 2 ? 3 : 0);
    printf("\nmulsub");
    put(a); put(e); put(c); put(d); put(fl_mul_sub(a, e, c, d));
    // |V| < 7p: k p + r with k in [-6, 5], r a product output, limbs scrambled
    Fl v = fl_mul(rnd_fl(0), rnd_fl(0));
    const int k = (int)(rnd() % 12) - 6;
    for (int i = 0; i < FL_N; i++) v.v[i] += k * (int32_t)FqParams::MOD28[i];
    for (int i = 0; i + 1 < FL_N; i++) {
      const int32_t s = (int32_t)(rnd() % 7) - 3;   // move s 2^28 from limb i+1 into limb i
      v.v[i] += s * (1 << 28);
      v.v[i + 1] -= s;
    }
    printf("\ncanon");
    put(v); put(fl_to_fq(v));
    Fl z = fl_zero();   // j p with scrambled limbs: must test zero
    const int j = (int)(rnd() % 13) - 6;
    for (int i = 0; i < FL_N; i++) z.v[i] = j * (int32_t)FqParams::MOD28[i];
    for (int i = 0; i + 1 < FL_N; i++) {
      const int32_t s = (int32_t)(rnd() % 5) - 2;
      z.v[i] += s * (1 << 28);
      z.v[i + 1] -= s;
    }
    printf("\nzero");
    put(z); printf(" %d", (int)fl_is_zero(z));
    put(v); printf(" %d\n", (int)fl_is_zero(v));
  }
  // the accumulate: acc += point i, the sign of the next point flipped where
  // the file asks (y given as p - y: a doubling or cancellation follows)
  FlX acc;
  flx_set_inf(acc);
  for (int i = 0; i < np; i++) {
    FlA a{fl_from_fq(pts[2 * i]), fl_from_fq(pts[2 * i + 1])};
    if (i % 3 == 1) a.y = fl_neg(fl_from_fq(pts[2 * i + 1]));   // negated as the kernel does (digit sign)
    acc = flx_madd(acc, a);
    printf("acc %d", i);
    put(fl_to_fq(acc.X)); put(fl_to_fq(acc.Y)); put(fl_to_fq(acc.ZZ)); put(fl_to_fq(acc.ZZZ));
    printf("\n");
  }
  return 0;
}
