// libnip.so -- variables and variable lists (src/nipvariable.h, declared in
// include/compat/nipvariable.h).
//
// Semantics of src/nipvariable.c: IDs come from one process-wide counter
// starting at NIP_VAR_MIN_ID (:60, shared with parse_model here, see
// nipamd_compat_take_ids); texts are copied and cut at NIP_VAR_TEXT_LENGTH
// bytes (:33-53); likelihoods start at 1 (:124-125); set operations keep the
// order of their first argument (union :446-503, isect :506-557); nip_mapper
// gives the position of each subset variable in the set (:560-589).
#include <cerrno>
#include <cstdlib>
#include <cstring>

#include "niperrorhandler.h"
#include "nipvariable.h"

namespace {

#define REPORT(e) nip_report_error((char*)__FILE__, __LINE__, (e), 1)

unsigned long g_next_id = NIP_VAR_MIN_ID;

// malloc'd copy of s cut at NIP_VAR_TEXT_LENGTH bytes (NULL for NULL)
char* text_copy(const char* s) {
  if (!s) return nullptr;
  size_t n = std::strlen(s);
  if (n > NIP_VAR_TEXT_LENGTH) n = NIP_VAR_TEXT_LENGTH;
  char* r = (char*)std::calloc(n + 1, 1);
  if (!r) {
    REPORT(ENOMEM);
    return nullptr;
  }
  std::memcpy(r, s, n);
  return r;
}

bool contains(nip_variable* a, int n, nip_variable v) {
  for (int i = 0; i < n; i++)
    if (nip_equal_variables(a[i], v)) return true;
  return false;
}

}  // namespace

extern "C" {

// reserve n consecutive IDs (parse_model numbers a model's variables from the
// same counter as nip_new_variable, like the reference's parser does)
unsigned long nipamd_compat_take_ids(int n) {
  const unsigned long first = g_next_id;
  g_next_id += (unsigned long)(n > 0 ? n : 0);
  return first;
}

nip_variable nip_new_variable(const char* symbol, const char* name, char** states, int cardinality) {
  auto* v = (nip_variable)std::calloc(1, sizeof(nip_variable_struct));
  if (!v) {
    REPORT(ENOMEM);
    return nullptr;
  }
  v->cardinality = cardinality;
  v->id = g_next_id++;
  v->interface_status = NIP_INTERFACE_NONE;
  v->pos_x = v->pos_y = 100;
  v->mark = NIP_MARK_OFF;
  v->symbol = text_copy(symbol);
  v->name = text_copy(name);  // may stay NULL, as in the reference (:90-93)
  if (states) {
    v->state_names = (char**)std::calloc(cardinality > 0 ? cardinality : 1, sizeof(char*));
    for (int i = 0; v->state_names && i < cardinality; i++) v->state_names[i] = text_copy(states[i]);
  } else {
    REPORT(EFAULT);  // nipvariable.c:112-113: reported, the variable is still made
  }
  v->likelihood = (double*)std::malloc(sizeof(double) * (cardinality > 0 ? cardinality : 1));
  if (!v->likelihood) {
    REPORT(ENOMEM);
    nip_free_variable(v);
    return nullptr;
  }
  for (int i = 0; i < cardinality; i++) v->likelihood[i] = 1.0;
  return v;
}

// the reference copies id, name, parents, family clique and likelihood only
// (:132-180); the rest of the record is left empty here
nip_variable nip_copy_variable(nip_variable v) {
  if (!v) return nullptr;
  auto* c = (nip_variable)std::calloc(1, sizeof(nip_variable_struct));
  if (!c) {
    REPORT(ENOMEM);
    return nullptr;
  }
  c->cardinality = v->cardinality;
  c->id = v->id;
  c->name = text_copy(v->name);
  c->num_of_parents = v->num_of_parents;
  if (v->parents && v->num_of_parents > 0) {
    c->parents = (nip_variable*)std::calloc(v->num_of_parents, sizeof(nip_variable));
    if (!c->parents) {
      REPORT(ENOMEM);
      nip_free_variable(c);
      return nullptr;
    }
    std::memcpy(c->parents, v->parents, sizeof(nip_variable) * v->num_of_parents);
  }
  c->family_clique = v->family_clique;
  c->likelihood = (double*)std::calloc(v->cardinality > 0 ? v->cardinality : 1, sizeof(double));
  if (!c->likelihood) {
    REPORT(ENOMEM);
    nip_free_variable(c);
    return nullptr;
  }
  std::memcpy(c->likelihood, v->likelihood, sizeof(double) * v->cardinality);
  return c;
}

void nip_free_variable(nip_variable v) {
  if (!v) return;
  std::free(v->symbol);
  std::free(v->name);
  if (v->state_names)
    for (int i = 0; i < v->cardinality; i++) std::free(v->state_names[i]);
  std::free(v->state_names);
  std::free(v->parents);
  std::free(v->family_mapping);
  std::free(v->likelihood);
  std::free(v->prior);
  std::free(v);
}

int nip_equal_variables(nip_variable v1, nip_variable v2) { return v1 && v2 ? v1->id == v2->id : 0; }
unsigned long nip_variable_id(nip_variable v) { return v ? v->id : 0; }
void nip_mark_variable(nip_variable v) { if (v) v->mark = NIP_MARK_ON; }
void nip_unmark_variable(nip_variable v) { if (v) v->mark = NIP_MARK_OFF; }
int nip_variable_marked(nip_variable v) { return v ? v->mark != NIP_MARK_OFF : 0; }
char* nip_variable_symbol(nip_variable v) { return v ? v->symbol : nullptr; }

int nip_variable_state_index(nip_variable v, char* state) {
  if (!v->state_names) return -1;
  for (int i = 0; i < v->cardinality; i++)
    if (std::strcmp(state, v->state_names[i]) == 0) return i;
  return -1;
}

char* nip_variable_state_name(nip_variable v, int index) {
  return v->state_names ? v->state_names[index] : nullptr;
}

nip_variable nip_search_variable_array(nip_variable* vars, int nvars, char* symbol) {
  for (int i = 0; i < nvars; i++)
    if (std::strcmp(symbol, vars[i]->symbol) == 0) return vars[i];
  return nullptr;
}

int nip_update_likelihood(nip_variable v, double likelihood[]) {
  if (!v || !likelihood) return REPORT(EFAULT);
  std::memcpy(v->likelihood, likelihood, sizeof(double) * v->cardinality);
  return 0;
}

void nip_reset_likelihood(nip_variable v) {
  if (!v) {
    REPORT(EFAULT);
    return;
  }
  for (int i = 0; i < v->cardinality; i++) v->likelihood[i] = 1.0;
}

int nip_number_of_parents(nip_variable v) {
  if (!v) {
    REPORT(EFAULT);
    return -1;
  }
  return v->num_of_parents;
}

void nip_set_variable_position(nip_variable v, int x, int y) {
  if (!v) {
    REPORT(EFAULT);
    return;
  }
  v->pos_x = x;
  v->pos_y = y;
}

void nip_get_variable_position(nip_variable v, int* x, int* y) {
  if (!(v && x && y)) {
    REPORT(EFAULT);
    return;
  }
  *x = v->pos_x;
  *y = v->pos_y;
}

int nip_set_parents(nip_variable v, nip_variable* parents, int nparents) {
  if (!v || (nparents > 0 && !parents)) return REPORT(EFAULT);
  std::free(v->parents);
  v->parents = nullptr;
  if (nparents > 0) {
    v->parents = (nip_variable*)std::calloc(nparents, sizeof(nip_variable));
    if (!v->parents) return REPORT(ENOMEM);
    std::memcpy(v->parents, parents, sizeof(nip_variable) * nparents);
  }
  v->num_of_parents = nparents;
  return 0;
}

nip_variable* nip_get_parents(nip_variable v) {
  if (!v) {
    REPORT(EFAULT);
    return nullptr;
  }
  return v->parents;
}

int nip_variable_is_parent(nip_variable parent, nip_variable child) {
  if (!parent || !child) return 0;
  return contains(child->parents, child->num_of_parents, parent) ? 1 : 0;
}

int nip_set_prior(nip_variable v, double* prior) {
  if (!v) return REPORT(EFAULT);
  if (!prior) return 0;  // nipvariable.c:389-390
  double* p = (double*)std::calloc(v->cardinality > 0 ? v->cardinality : 1, sizeof(double));
  if (!p) return REPORT(ENOMEM);
  std::memcpy(p, prior, sizeof(double) * v->cardinality);
  std::free(v->prior);
  v->prior = p;
  return 0;
}

double* nip_get_prior(nip_variable v) {
  if (!v) {
    REPORT(EFAULT);
    return nullptr;
  }
  return v->prior;
}

// The reference's exchange loop (:427-440): for every position i < n-1 the
// inner index restarts at 1, not i+1, so for n >= 4 the result is not always
// ascending (IDs 4,3,2,1 give 1,4,2,3).  The same exchanges are made here so
// callers get the reference's array.
nip_variable* nip_sort_variables(nip_variable* vars, int nvars) {
  if (nvars < 1) {
    REPORT(EINVAL);
    return nullptr;
  }
  auto* s = (nip_variable*)std::calloc(nvars, sizeof(nip_variable));
  if (!s) {
    REPORT(ENOMEM);
    return nullptr;
  }
  std::memcpy(s, vars, sizeof(nip_variable) * nvars);
  for (int i = 0; i + 1 < nvars; i++)
    for (int j = 1; j < nvars; j++)
      if (s[j]->id < s[i]->id) {
        nip_variable t = s[j];
        s[j] = s[i];
        s[i] = t;
      }
  return s;
}

nip_variable* nip_variable_union(nip_variable* a, nip_variable* b, int na, int nb, int* nc) {
  if (!nc || (na > 0 && !a) || (nb > 0 && !b)) {
    REPORT(EFAULT);
    if (nc) *nc = -1;
    return nullptr;
  }
  if (na <= 0 && nb <= 0) {
    *nc = 0;
    return nullptr;
  }
  int n = na > 0 ? na : 0;
  for (int i = 0; i < nb; i++)
    if (!contains(a, na, b[i])) n++;
  *nc = n;
  if (n == 0) return nullptr;
  auto* c = (nip_variable*)std::calloc(n, sizeof(nip_variable));
  if (!c) {
    REPORT(ENOMEM);
    *nc = -1;
    return nullptr;
  }
  int k = 0;
  for (int i = 0; i < na; i++) c[k++] = a[i];
  for (int i = 0; i < nb; i++)
    if (!contains(c, k, b[i])) c[k++] = b[i];
  return c;
}

nip_variable* nip_variable_isect(nip_variable* a, nip_variable* b, int na, int nb, int* nc) {
  if (na == 0 || nb == 0) {
    if (nc) *nc = 0;
    return nullptr;
  }
  if (!a || !b) {
    REPORT(EFAULT);
    if (nc) *nc = -1;
    return nullptr;
  }
  int n = 0;
  for (int i = 0; i < na; i++)
    if (contains(b, nb, a[i])) n++;
  *nc = n;
  if (n == 0) return nullptr;
  auto* c = (nip_variable*)std::calloc(n, sizeof(nip_variable));
  if (!c) {
    REPORT(ENOMEM);
    *nc = -1;
    return nullptr;
  }
  int k = 0;
  for (int i = 0; i < na; i++)
    if (contains(b, nb, a[i])) c[k++] = a[i];
  return c;
}

int* nip_mapper(nip_variable* set, nip_variable* subset, int nset, int nsubset) {
  if (nsubset < 1) return nullptr;
  if (!(set && subset && nset >= nsubset)) {
    REPORT(EINVAL);
    return nullptr;
  }
  int* m = (int*)std::calloc(nsubset, sizeof(int));
  if (!m) {
    REPORT(ENOMEM);
    return nullptr;
  }
  for (int i = 0; i < nsubset; i++)
    for (int j = 0; j < nset; j++)
      if (nip_equal_variables(subset[i], set[j])) {
        m[i] = j;
        break;
      }
  return m;
}

/* ---- variable and interface lists (nipvariable.c:592-821) ---- */

nip_variable_list nip_new_variable_list(void) {
  auto* l = (nip_variable_list)std::calloc(1, sizeof(nip_variable_list_struct));
  if (!l) REPORT(ENOMEM);
  return l;
}

nip_interface_list nip_new_interface_list(void) {
  auto* l = (nip_interface_list)std::calloc(1, sizeof(nip_iflist_struct));
  if (!l) REPORT(ENOMEM);
  return l;
}

}  // extern "C"

namespace {
template <class List, class Link>
void link_in(List* l, Link* k, bool front) {
  if (front) {
    k->bwd = nullptr;
    k->fwd = l->first;
    if (l->first) l->first->bwd = k; else l->last = k;
    l->first = k;
  } else {
    k->fwd = nullptr;
    k->bwd = l->last;
    if (l->last) l->last->fwd = k; else l->first = k;
    l->last = k;
  }
  l->length++;
}

int add_variable(nip_variable_list l, nip_variable v, bool front) {
  if (!l || !v) return REPORT(EFAULT);
  auto* k = (nip_variable_link)std::malloc(sizeof(nip_variable_link_struct));
  if (!k) return REPORT(ENOMEM);
  k->data = v;
  link_in(l, k, front);
  return 0;
}

int add_interface(nip_interface_list l, nip_variable var, char* next, bool front) {
  if (!l || !var) return REPORT(EFAULT);
  auto* k = (nip_interface_link)std::malloc(sizeof(nip_iflink_struct));
  if (!k) return REPORT(ENOMEM);
  k->var = var;
  k->next = next;  // the list owns the string (nipvariable.c:647-648)
  link_in(l, k, front);
  return 0;
}
}  // namespace

extern "C" {

int nip_append_variable(nip_variable_list l, nip_variable v) { return add_variable(l, v, false); }
int nip_prepend_variable(nip_variable_list l, nip_variable v) { return add_variable(l, v, true); }
int nip_append_interface(nip_interface_list l, nip_variable var, char* next) {
  return add_interface(l, var, next, false);
}
int nip_prepend_interface(nip_interface_list l, nip_variable var, char* next) {
  return add_interface(l, var, next, true);
}

nip_variable* nip_variable_list_to_array(nip_variable_list l) {
  if (!l) {
    REPORT(EFAULT);
    return nullptr;
  }
  if (l->length == 0) return nullptr;
  auto* a = (nip_variable*)std::calloc(l->length, sizeof(nip_variable));
  if (!a) {
    REPORT(ENOMEM);
    return nullptr;
  }
  int i = 0;
  for (nip_variable_link k = l->first; k && i < l->length; k = k->fwd) a[i++] = k->data;
  return a;
}

void nip_empty_variable_list(nip_variable_list l) {
  if (!l) return;
  for (nip_variable_link k = l->first; k;) {
    nip_variable_link n = k->fwd;
    std::free(k);
    k = n;
  }
  l->first = l->last = nullptr;
  l->length = 0;
}

void nip_free_interface_list(nip_interface_list l) {
  if (!l) return;
  for (nip_interface_link k = l->first; k;) {
    nip_interface_link n = k->fwd;
    std::free(k->next);
    std::free(k);
    k = n;
  }
  std::free(l);
}

nip_variable nip_next_variable(nip_variable_iterator* it) {
  if (!*it) return nullptr;
  nip_variable v = (*it)->data;
  *it = (*it)->fwd;
  return v;
}

nip_variable nip_search_variable_list(nip_variable_list l, char* symbol) {
  for (nip_variable_link k = l->first; k; k = k->fwd)
    if (std::strcmp(symbol, nip_variable_symbol(k->data)) == 0) return k->data;
  return nullptr;
}

}  // extern "C"
