/*
 * nipparsers.h -- the reference's src/nipparsers.h data-file bookkeeping
 * struct and constants (nipparsers.h:27-66), so code that includes it
 * (util/nipjoint.c:39, and nip.h itself, nip.h:39) compiles against the
 * nip_amd compat layer.  The data-file reader of this layer is
 * read_timeseries / write_timeseries in nip.h (nip_amd/csrc/datafile.cpp
 * restates nipparsers.c's tokenizer); the low-level nip_open_data_file /
 * nip_next_line_tokens / nip_next_hugin_token entry points are not exported,
 * so a caller of those fails at compile time rather than at run time.
 */
#ifndef NIP_AMD_COMPAT_PARSERS_H
#define NIP_AMD_COMPAT_PARSERS_H

#include <stdio.h>

#define MAX_LINELENGTH 10000
#define NIP_COMMENT_CHAR '%'

typedef struct {
  char* name;
  char separator;
  FILE* file;
  int is_open;
  int first_line_labels;
  int current_line;
  int label_line;
  int ndatarows;
  int* datarows;
  int num_of_nodes;
  char** node_symbols;
  int* num_of_states;
  char*** node_states;
} nip_data_file_struct;

typedef nip_data_file_struct* nip_data_file;

#endif
