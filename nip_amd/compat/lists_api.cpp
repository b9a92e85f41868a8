// libnip.so -- the reference's linked lists (src/niplists.h, declared in
// include/compat/niplists.h).  Every list type is a doubly linked list with
// the same (length, first, last) header and (payload..., fwd, bwd) links, so
// the operations are written once as templates over the link type.
//
// Behaviour follows src/niplists.c: append/prepend report EFAULT on a NULL
// list (string pairs also on a NULL key or value, :207-209) and ENOMEM when a
// link cannot be allocated; *_to_array returns NULL for an empty list
// (:385-386, :413-414) with the payload copied (strings by pointer); empty_*
// frees the links only; free_* frees the payloads it owns and the list.
#include <cerrno>
#include <cstdlib>
#include <cstring>
#include <type_traits>

#include "niperrorhandler.h"
#include "niplists.h"

namespace {

#define REPORT(e) nip_report_error((char*)__FILE__, __LINE__, (e), 1)

template <class List>
List* new_list() {
  auto* l = (List*)std::malloc(sizeof(List));
  if (!l) {
    REPORT(ENOMEM);
    return nullptr;
  }
  l->length = 0;
  l->first = l->last = nullptr;
  return l;
}

// link a new element at the end (front = false) or the beginning
template <class List, class Fill>
int insert(List* l, bool front, Fill fill) {
  using Link = std::remove_pointer_t<decltype(l->first)>;
  if (!l) return REPORT(EFAULT);
  auto* k = (Link*)std::malloc(sizeof(Link));
  if (!k) return REPORT(ENOMEM);
  fill(k);
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
  return 0;
}

// free every link, calling drop(link) first
template <class List, class Drop>
void unlink_all(List* l, Drop drop) {
  if (!l) return;
  for (auto* k = l->first; k;) {
    auto* n = k->fwd;
    drop(k);
    std::free(k);
    k = n;
  }
  l->first = l->last = nullptr;
  l->length = 0;
}

template <class T, class List>
T* to_array(List* l) {
  if (!l) {
    REPORT(EFAULT);
    return nullptr;
  }
  if (l->length == 0) return nullptr;
  auto* a = (T*)std::calloc(l->length, sizeof(T));
  if (!a) {
    REPORT(ENOMEM);
    return nullptr;
  }
  int i = 0;
  for (auto* k = l->first; k && i < l->length; k = k->fwd) a[i++] = k->data;
  return a;
}

const auto keep = [](auto*) {};

}  // namespace

extern "C" {

nip_int_array_list nip_new_int_array_list(void) { return new_list<nip_int_array_list_struct>(); }
nip_int_list nip_new_int_list(void) { return new_list<nip_int_list_struct>(); }
nip_double_list nip_new_double_list(void) { return new_list<nip_double_list_struct>(); }
nip_string_list nip_new_string_list(void) { return new_list<nip_string_list_struct>(); }
nip_string_pair_list nip_new_string_pair_list(void) { return new_list<nip_string_pair_list_struct>(); }

int nip_append_int_array(nip_int_array_list l, int* i, int ni) {
  return insert(l, false, [&](nip_int_array_link k) { k->data = i; k->size = ni; });
}
int nip_prepend_int_array(nip_int_array_list l, int* i, int ni) {
  return insert(l, true, [&](nip_int_array_link k) { k->data = i; k->size = ni; });
}
int nip_append_int(nip_int_list l, int i) {
  return insert(l, false, [&](nip_int_link k) { k->data = i; });
}
int nip_prepend_int(nip_int_list l, int i) {
  return insert(l, true, [&](nip_int_link k) { k->data = i; });
}
int nip_append_double(nip_double_list l, double d) {
  return insert(l, false, [&](nip_double_link k) { k->data = d; });
}
int nip_prepend_double(nip_double_list l, double d) {
  return insert(l, true, [&](nip_double_link k) { k->data = d; });
}
int nip_append_string(nip_string_list l, char* s) {
  return insert(l, false, [&](nip_string_link k) { k->data = s; });
}
int nip_prepend_string(nip_string_list l, char* s) {
  return insert(l, true, [&](nip_string_link k) { k->data = s; });
}
int nip_append_string_pair(nip_string_pair_list l, char* key, char* value) {
  if (!key || !value) return REPORT(EFAULT);
  return insert(l, false, [&](nip_string_pair_link k) { k->key = key; k->value = value; });
}
int nip_prepend_string_pair(nip_string_pair_list l, char* key, char* value) {
  if (!key || !value) return REPORT(EFAULT);
  return insert(l, true, [&](nip_string_pair_link k) { k->key = key; k->value = value; });
}

int* nip_int_list_to_array(nip_int_list l) { return to_array<int>(l); }
double* nip_double_list_to_array(nip_double_list l) { return to_array<double>(l); }
char** nip_string_list_to_array(nip_string_list l) { return to_array<char*>(l); }

void nip_empty_int_array_list(nip_int_array_list l) { unlink_all(l, keep); }
void nip_empty_int_list(nip_int_list l) { unlink_all(l, keep); }
void nip_empty_double_list(nip_double_list l) { unlink_all(l, keep); }
void nip_empty_string_list(nip_string_list l) { unlink_all(l, keep); }

void nip_free_int_array_list(nip_int_array_list l) {
  unlink_all(l, [](nip_int_array_link k) { std::free(k->data); });
  std::free(l);
}
void nip_free_string_list(nip_string_list l) {
  unlink_all(l, [](nip_string_link k) { std::free(k->data); });
  std::free(l);
}
void nip_free_string_pair_list(nip_string_pair_list l) {
  unlink_all(l, [](nip_string_pair_link k) { std::free(k->key); std::free(k->value); });
  std::free(l);
}

// true if some array of the list is a superset of the indicator vector i
// (niplists.c:598-619: i[v] set and lnk->data[v] clear disqualifies lnk)
int nip_int_array_list_contains_subset(nip_int_array_list l, int* i, int ni) {
  if (!l) return 0;
  for (nip_int_array_link k = l->first; k; k = k->fwd) {
    bool sub = true;
    for (int v = 0; v < ni && sub; v++) sub = !(i[v] && !k->data[v]);
    if (sub) return 1;
  }
  return 0;
}

int nip_string_list_contains(nip_string_list l, char* string) {
  if (!l || !string) return 0;
  for (nip_string_link k = l->first; k; k = k->fwd)
    if (std::strcmp(string, k->data) == 0) return 1;
  return 0;
}

char* nip_string_pair_list_search(nip_string_pair_list l, char* key) {
  if (!l || !key) return nullptr;
  for (nip_string_pair_link k = l->first; k; k = k->fwd)
    if (std::strcmp(key, k->key) == 0) return k->value;
  return nullptr;
}

}  // extern "C"
