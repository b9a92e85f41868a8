/*
 * slice_driver.c -- TEST INFRASTRUCTURE ONLY.
 *
 * Runs a single-slice script (oracle/ref/slice_script.h) against libnip.so
 * through the compat headers (include/compat/nip.h): reset_model, use_priors,
 * make_consistent (GPU Hugin propagation), nip_collect_evidence /
 * nip_distribute_evidence, get_probability, get_joint_probability.  The
 * harness runs the same script over the reference's own code (nh_slice);
 * tests/test_gpu_slice.py compares the two outputs bit for bit.
 *
 * usage: slice_driver MODEL.NET SCRIPT
 */
#include <stdio.h>
#include "nip.h"

#define SS_MODEL nip_model
#define SS_RESET(m) reset_model(m)
#define SS_PRIORS(m, h) use_priors(m, h)
#define SS_CONSISTENT(m) make_consistent(m)
#define SS_PROB(m, v) get_probability(m, v)
#define SS_JOINT(m, vs, n) get_joint_probability(m, vs, n)
#define ss_put(ctx, ...) fprintf((FILE*)(ctx), __VA_ARGS__)
#include "slice_script.h"

int main(int argc, char** argv){
  nip_model m;
  int rc;
  if(argc < 3){
    fprintf(stderr, "usage: %s MODEL.NET SCRIPT\n", argv[0]);
    return 2;
  }
  m = parse_model(argv[1]);
  if(!m) return 1;
  rc = ss_run(stdout, m, argv[2]);
  free_model(m);
  return rc ? 3 : 0;
}
