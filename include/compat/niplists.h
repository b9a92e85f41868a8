/*
 * niplists.h -- drop-in for the reference's src/niplists.h (nip_amd compat
 * layer, libnip.so): the linked lists of ints, int arrays, doubles, strings
 * and key/value string pairs, in the layouts of niplists.h:30-127 (callers
 * walk first/fwd/bwd/data directly, e.g. util/niptrain.c:173-199 over the
 * learning curve; every potential owns a string-pair list,
 * nippotential.h:54).  Implemented in nip_amd/compat/lists_api.cpp.
 *
 * Ownership follows the reference: string and string-pair lists store the
 * caller's pointers and free them in nip_free_*_list (niplists.c:538-595);
 * int arrays are freed by nip_free_int_array_list.
 */
#ifndef NIP_AMD_COMPAT_LISTS_H
#define NIP_AMD_COMPAT_LISTS_H

#ifdef __cplusplus
extern "C" {
#endif

#define NIP_LIST_LENGTH(l) ((l)->length)

typedef struct nip_int_array_link_type {
  int* data;
  int size;
  struct nip_int_array_link_type* fwd;
  struct nip_int_array_link_type* bwd;
} nip_int_array_link_struct;
typedef nip_int_array_link_struct* nip_int_array_link;

typedef struct nip_int_array_list_type {
  int length;
  nip_int_array_link first;
  nip_int_array_link last;
} nip_int_array_list_struct;
typedef nip_int_array_list_struct* nip_int_array_list;

typedef struct nip_int_link_type {
  int data;
  struct nip_int_link_type* fwd;
  struct nip_int_link_type* bwd;
} nip_int_link_struct;
typedef nip_int_link_struct* nip_int_link;

typedef struct nip_int_list_type {
  int length;
  nip_int_link first;
  nip_int_link last;
} nip_int_list_struct;
typedef nip_int_list_struct* nip_int_list;

typedef struct nip_double_link_type {
  double data;
  struct nip_double_link_type* fwd;
  struct nip_double_link_type* bwd;
} nip_double_link_struct;
typedef nip_double_link_struct* nip_double_link;

typedef struct nip_double_list_type {
  int length;
  nip_double_link first;
  nip_double_link last;
} nip_double_list_struct;
typedef nip_double_list_struct* nip_double_list;

typedef struct nip_string_link_type {
  char* data;
  struct nip_string_link_type* fwd;
  struct nip_string_link_type* bwd;
} nip_string_link_struct;
typedef nip_string_link_struct* nip_string_link;

typedef struct nip_string_list_type {
  int length;
  nip_string_link first;
  nip_string_link last;
} nip_string_list_struct;
typedef nip_string_list_struct* nip_string_list;

typedef struct nip_string_pair_link_type {
  char* key;
  char* value;
  struct nip_string_pair_link_type* fwd;
  struct nip_string_pair_link_type* bwd;
} nip_string_pair_link_struct;
typedef nip_string_pair_link_struct* nip_string_pair_link;

typedef struct nip_string_pair_list_type {
  int length;
  nip_string_pair_link first;
  nip_string_pair_link last;
} nip_string_pair_list_struct;
typedef nip_string_pair_list_struct* nip_string_pair_list;

nip_int_array_list nip_new_int_array_list(void);
nip_int_list nip_new_int_list(void);
nip_double_list nip_new_double_list(void);
nip_string_list nip_new_string_list(void);
nip_string_pair_list nip_new_string_pair_list(void);

int nip_append_int_array(nip_int_array_list l, int* i, int ni);
int nip_append_int(nip_int_list l, int i);
int nip_append_double(nip_double_list l, double d);
int nip_append_string(nip_string_list l, char* s);
int nip_append_string_pair(nip_string_pair_list l, char* key, char* value);

int nip_prepend_int_array(nip_int_array_list l, int* i, int ni);
int nip_prepend_int(nip_int_list l, int i);
int nip_prepend_double(nip_double_list l, double d);
int nip_prepend_string(nip_string_list l, char* s);
int nip_prepend_string_pair(nip_string_pair_list l, char* key, char* value);

int* nip_int_list_to_array(nip_int_list l);          /* malloc'd; NULL if empty */
double* nip_double_list_to_array(nip_double_list l); /* malloc'd; NULL if empty */
char** nip_string_list_to_array(nip_string_list l);  /* malloc'd; the strings are shared */

void nip_empty_int_array_list(nip_int_array_list l); /* frees the links, not l */
void nip_empty_int_list(nip_int_list l);
void nip_empty_double_list(nip_double_list l);
void nip_empty_string_list(nip_string_list l);

void nip_free_int_array_list(nip_int_array_list l);  /* frees the arrays too */
void nip_free_string_list(nip_string_list l);        /* frees the strings too */
void nip_free_string_pair_list(nip_string_pair_list l);

int nip_int_array_list_contains_subset(nip_int_array_list l, int* i, int ni);
int nip_string_list_contains(nip_string_list l, char* string);
char* nip_string_pair_list_search(nip_string_pair_list l, char* key);

#ifdef __cplusplus
}
#endif
#endif
