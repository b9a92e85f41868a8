/*
 * nipvariable.h -- drop-in for the reference's src/nipvariable.h (nip_amd
 * compat layer, libnip.so): the variable record with the field order and
 * types of nipvariable.h:51-78, so code that reads fields directly keeps
 * working, and the accessors the time-series API's callers use.  The join
 * tree lives in the GPU engine, so family_clique / family_mapping are NULL.
 */
#ifndef NIP_AMD_COMPAT_VARIABLE_H
#define NIP_AMD_COMPAT_VARIABLE_H

#ifdef __cplusplus
extern "C" {
#endif

#define NIP_VAR_TEXT_LENGTH 40
#define NIP_VAR_MIN_ID      1
#define NIP_VAR_INVALID_ID  0

/* interface roles in a DBN slice (bit flags) */
#define NIP_INTERFACE_NONE          0
#define NIP_INTERFACE_INCOMING      1
#define NIP_INTERFACE_OUTGOING      (1 << 1)
#define NIP_INTERFACE_OLD_OUTGOING  (1 << 2)

/* marks: only marked variables' evidence is entered (src/nip.c:993) */
#define NIP_MARK_OFF   1
#define NIP_MARK_ON    (1 << 1)
#define NIP_MARK_BOTH  (NIP_MARK_OFF | NIP_MARK_ON)

#define NIP_CARDINALITY(v) ((v)->cardinality)
#define NIP_MARK(v)        ((v)->mark)
#define NIP_IF(v)          ((v)->interface_status)

typedef struct nip_var {
  unsigned long id;          /* 1, 2, ... in declaration order */
  char* symbol;
  char* name;                /* the .net label */
  int cardinality;
  char** state_names;
  double* likelihood;
  double* prior;             /* independent variables only, else NULL */
  int prior_entered;
  struct nip_var* previous;  /* this variable in the previous slice */
  struct nip_var* next;      /* this variable in the next slice (NIP_next) */
  int num_of_parents;
  struct nip_var** parents;
  void* family_clique;       /* NULL: the join tree is the engine's */
  int* family_mapping;       /* NULL */
  int interface_status;
  char mark;
  int pos_x;
  int pos_y;
} nip_variable_struct;

typedef nip_variable_struct* nip_variable;

void nip_mark_variable(nip_variable v);
void nip_unmark_variable(nip_variable v);
int nip_variable_marked(nip_variable v);
char* nip_variable_symbol(nip_variable v);
int nip_variable_state_index(nip_variable v, char* state);
char* nip_variable_state_name(nip_variable v, int index);
int nip_equal_variables(nip_variable v1, nip_variable v2);
int nip_number_of_parents(nip_variable v);

#ifdef __cplusplus
}
#endif
#endif
