/*
 * nipvariable.h -- drop-in for the reference's src/nipvariable.h (nip_amd
 * compat layer, libnip.so): the variable record with the field order and
 * types of nipvariable.h:51-78, so code that reads fields directly keeps
 * working, the variable / interface lists of :84-124, and every function of
 * :134-413 (nip_amd/compat/variable_api.cpp).  Variables of a parsed model
 * are owned by the model (free_model); nip_new_variable creates free-standing
 * ones for callers that build join trees by hand (test/cliquetest.c).
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
  unsigned long id;          /* 1, 2, ... in creation order */
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
  void* family_clique;       /* memo of nip_find_family (a nip_clique) */
  int* family_mapping;       /* memo of nip_find_family_mapping */
  int interface_status;
  char mark;
  int pos_x;
  int pos_y;
} nip_variable_struct;

typedef nip_variable_struct* nip_variable;

typedef struct nip_varlink {
  nip_variable data;
  struct nip_varlink* fwd;
  struct nip_varlink* bwd;
} nip_variable_link_struct;
typedef nip_variable_link_struct* nip_variable_link;
typedef nip_variable_link nip_variable_iterator;

typedef struct nip_varlist {
  int length;
  nip_variable_link first;
  nip_variable_link last;
} nip_variable_list_struct;
typedef nip_variable_list_struct* nip_variable_list;

typedef struct nip_iflink {
  nip_variable var;
  char* next;
  struct nip_iflink* fwd;
  struct nip_iflink* bwd;
} nip_iflink_struct;
typedef nip_iflink_struct* nip_interface_link;

typedef struct nip_iflist {
  int length;
  nip_interface_link first;
  nip_interface_link last;
} nip_iflist_struct;
typedef nip_iflist_struct* nip_interface_list;

nip_variable nip_new_variable(const char* symbol, const char* name, char** states, int cardinality);
nip_variable nip_copy_variable(nip_variable v);
void nip_free_variable(nip_variable v);
int nip_equal_variables(nip_variable v1, nip_variable v2);
unsigned long nip_variable_id(nip_variable v);
void nip_mark_variable(nip_variable v);
void nip_unmark_variable(nip_variable v);
int nip_variable_marked(nip_variable v);
char* nip_variable_symbol(nip_variable v);
int nip_variable_state_index(nip_variable v, char* state);
char* nip_variable_state_name(nip_variable v, int index);
nip_variable nip_search_variable_array(nip_variable* vars, int nvars, char* symbol);
int nip_update_likelihood(nip_variable v, double likelihood[]);
void nip_reset_likelihood(nip_variable v);
int nip_number_of_parents(nip_variable v);
void nip_set_variable_position(nip_variable v, int x, int y);
void nip_get_variable_position(nip_variable v, int* x, int* y);
int nip_set_parents(nip_variable v, nip_variable* parents, int nparents);
nip_variable* nip_get_parents(nip_variable v);
int nip_variable_is_parent(nip_variable parent, nip_variable child);
int nip_set_prior(nip_variable v, double* prior);
double* nip_get_prior(nip_variable v);
nip_variable* nip_sort_variables(nip_variable* vars, int nvars);
nip_variable* nip_variable_union(nip_variable* a, nip_variable* b, int na, int nb, int* nc);
nip_variable* nip_variable_isect(nip_variable* a, nip_variable* b, int na, int nb, int* nc);
int* nip_mapper(nip_variable* set, nip_variable* subset, int nset, int nsubset);

nip_variable_list nip_new_variable_list(void);
nip_interface_list nip_new_interface_list(void);
int nip_append_variable(nip_variable_list l, nip_variable v);
int nip_append_interface(nip_interface_list l, nip_variable var, char* next);
int nip_prepend_variable(nip_variable_list l, nip_variable v);
int nip_prepend_interface(nip_interface_list l, nip_variable var, char* next);
nip_variable* nip_variable_list_to_array(nip_variable_list l);
void nip_empty_variable_list(nip_variable_list l);
void nip_free_interface_list(nip_interface_list l);
nip_variable nip_next_variable(nip_variable_iterator* it);
nip_variable nip_search_variable_list(nip_variable_list l, char* symbol);

#ifdef __cplusplus
}
#endif
#endif
