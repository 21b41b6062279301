// Host-side sanitizer harness: drives the native library's pure
// host code -- the launch planners that size every grid / split / workspace
// -- over the X-UNet's shapes at every per-GPU batch and over edge shapes,
// with the library's HOST code built under AddressSanitizer +
// UndefinedBehaviorSanitizer (tools/host_sanitize/run.sh).  GPU code is not
// instrumented (GPU sanitizers are not available on this pool) and no GPU is
// needed: the planners make no HIP calls.  Also checks planner invariants
// (splits cover the reduction, workspace sizes are positive and bounded).
#include <cstdio>
#include <cstdlib>

extern "C" {
int d3d_conv_plan(int N, int OH, int OW, int OC, int ICp, int taps);
int d3d_conv_wgrad_plan2(int N, int OH, int OW, int OC, int IC, int taps, int* splits, int* pix_per_split);
int d3d_conv_wgrad_plan3(int N, int IH, int IW, int OH, int OW, int OC, int IC, int taps, int stride, int* splits,
                         int* pix_per_split);
int d3d_gn_plan(int N, int P, int C, int* nchunks, int* rows);
}

static int fails = 0;
#define CHECK(c, ...)                       \
  do {                                      \
    if (!(c)) {                             \
      ++fails;                              \
      std::fprintf(stderr, __VA_ARGS__);    \
      std::fprintf(stderr, "\n");           \
    }                                       \
  } while (0)

int main() {
  const int batches[] = {1, 2, 3, 4, 8, 16, 32, 64, 128, 256};
  const int sizes[] = {4, 8, 16, 32, 64, 128};
  const int chans[] = {3, 8, 64, 128, 144, 256, 384, 512, 768, 1024, 1536, 4608};
  long checked = 0;
  for (int N : batches)
    for (int H : sizes)
      for (int OC : chans)
        for (int IC : chans) {
          const int ICp = (IC + 63) / 64 * 64;
          for (int taps : {1, 9}) {
            const int ns = d3d_conv_plan(N, H, H, OC, ICp, taps);
            CHECK(ns >= 1 && ns <= 16, "conv_plan N%d H%d OC%d IC%d taps%d -> %d", N, H, OC, IC, taps, ns);
            int sp = 0, pps = 0;
            d3d_conv_wgrad_plan2(N, H, H, OC, IC, taps, &sp, &pps);
            const long P = (long)N * H * H;
            CHECK(sp >= 1 && pps >= 1 && (long)sp * pps >= P && (long)(sp - 1) * pps < P && pps % 64 == 0,
                  "wgrad_plan2 N%d H%d OC%d IC%d taps%d -> %d x %d", N, H, OC, IC, taps, sp, pps);
            for (int stride : {1, 2}) {
              const int OH = (H - 1) / stride + 1;
              d3d_conv_wgrad_plan3(N, H, H, OH, OH, OC, IC, taps, stride, &sp, &pps);
              const long Po = (long)N * OH * OH;
              CHECK(sp >= 1 && pps >= 1 && (long)sp * pps >= Po && pps % 64 == 0,
                    "wgrad_plan3 N%d H%d s%d OC%d IC%d taps%d -> %d x %d", N, H, stride, OC, IC, taps, sp, pps);
            }
            ++checked;
          }
          if (OC % 8 == 0) {
            int nch = 0, rows = 0;
            d3d_gn_plan(N, H * H, OC, &nch, &rows);
            CHECK(nch >= 1 && rows >= 1 && (long)nch * rows >= (long)H * H, "gn_plan N%d P%d C%d -> %d x %d", N,
                  H * H, OC, nch, rows);
          }
        }
  std::printf("host planners: %ld shape combinations checked, %d invariant failures\n", checked, fails);
  return fails ? 1 : 0;
}
