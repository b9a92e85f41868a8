/*
 * niplists.h -- drop-in for the part of the reference's src/niplists.h the
 * time-series API uses: the list of doubles em_learn fills with the learning
 * curve (the layout of niplists.h:73-86; callers walk first/fwd/bwd/data
 * directly, util/niptrain.c:173-199).
 */
#ifndef NIP_AMD_COMPAT_LISTS_H
#define NIP_AMD_COMPAT_LISTS_H

#ifdef __cplusplus
extern "C" {
#endif

#define NIP_LIST_LENGTH(l) ((l)->length)

typedef struct nip_double_link_type {
  double data;
  struct nip_double_link_type* fwd;
  struct nip_double_link_type* bwd;
} nip_double_link_struct;
typedef nip_double_link_struct* nip_double_link;

typedef struct {
  int length;
  nip_double_link first;
  nip_double_link last;
} nip_double_list_struct;
typedef nip_double_list_struct* nip_double_list;

nip_double_list nip_new_double_list(void);
int nip_append_double(nip_double_list l, double d);
int nip_prepend_double(nip_double_list l, double d);
double* nip_double_list_to_array(nip_double_list l); /* malloc'd; NULL if empty */
void nip_empty_double_list(nip_double_list l);       /* frees the links, not l */

#ifdef __cplusplus
}
#endif
#endif
