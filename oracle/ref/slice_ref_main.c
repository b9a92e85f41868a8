/*
 * slice_ref_main.c -- TEST INFRASTRUCTURE ONLY (oracle).
 * usage: slice_ref REPLAY_FILE SCRIPT
 * Builds the model from a grammar replay (oracle/netfile.py) through the
 * reference's own code (libnipref.so, nh_build) and prints the slice script's
 * output (nh_slice, oracle/ref/slice_script.h).  A separate process, because
 * the reference's nip_gather_joint_probability corrupts its heap for some
 * variable sets (nipjointree.c:1372-1377 writes n_vars + n_isect
 * cardinalities into an array of nprod) and the tests must survive that.
 */
#include <stdio.h>
#include <stdlib.h>

int nh_build(const char* replay);
int nh_slice(int h, const char* script, char* buf, int cap);

int main(int argc, char** argv){
  FILE* f;
  long n;
  char* replay;
  char* out;
  int h, cap = 1 << 20, len;
  if(argc < 3) return 2;
  f = fopen(argv[1], "rb");
  if(!f) return 2;
  fseek(f, 0, SEEK_END); n = ftell(f); fseek(f, 0, SEEK_SET);
  replay = (char*) calloc(n + 1, 1);
  if(fread(replay, 1, n, f) != (size_t)n) return 2;
  fclose(f);
  h = nh_build(replay);
  if(h < 0) return 1;
  for(;;){
    out = (char*) malloc(cap);
    len = nh_slice(h, argv[2], out, cap);
    if(len < 0) return 3;
    if(len < cap) break;
    free(out);
    cap = len + 1;
  }
  fputs(out, stdout);
  return 0;
}
