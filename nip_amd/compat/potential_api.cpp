// libnip.so -- potentials (src/nippotential.h, declared in
// include/compat/nippotential.h) on caller-owned host tables.
//
// Every arithmetic operation is the reference's, in the reference's order
// (src/nippotential.c), so results are bit-identical:
//   general_marginalise (:267-311)  dest := 0, then dest[choose(i)] += src[i]
//                                   for i ascending (a scalar dest sums all)
//   update_potential    (:436-496)  t[i] *= num[j]; t[i] = den[j] ? t[i]/den[j] : 0
//   update_evidence     (:499-522)  t[i] *= num[k]; den[k] != 0 -> t[i] /= den[k]
//   init_potential      (:525-564)  t[i] *= probs[choose(i)] (elementwise without a
//                                   mapping; a scalar probs is a no-op)
//   normalise_array     (:349-359)  sum ascending, no-op on a zero sum
// Instead of an inverse mapping per element (integer divisions per dimension,
// the reference's hottest instructions) the loops walk the table with an
// odometer over the multi-index and carry the projected offset along.
#include <cerrno>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <vector>

#include "niperrorhandler.h"
#include "nippotential.h"

namespace {

#define REPORT(e) nip_report_error((char*)__FILE__, __LINE__, (e), 1)

// Walks the entries of `big` in flat order and keeps, for each, the flat
// offset of its projection onto a smaller table whose dimension k is big's
// dimension map[k] (map[k] = -1: not projected).  step(i, j) is called for
// every flat index i with projected offset j.
template <class Step>
void walk_projection(const nip_potential big, const int* map, int nmap, const int* small_card,
                     Step step) {
  const int d = big->dimensionality;
  std::vector<long> stride(d > 0 ? d : 1, 0);   // projected stride of each big dimension
  long s = 1;
  for (int k = 0; k < nmap; k++) {
    if (map[k] >= 0 && map[k] < d) stride[map[k]] += s;
    s *= small_card[k];
  }
  std::vector<int> idx(d > 0 ? d : 1, 0);
  long j = 0;
  for (int i = 0; i < big->size_of_data; i++) {
    step(i, j);
    for (int a = 0; a < d; a++) {       // odometer, dimension 0 fastest
      j += stride[a];
      if (++idx[a] < big->cardinality[a]) break;
      j -= stride[a] * idx[a];
      idx[a] = 0;
    }
  }
}

bool same_geometry(const nip_potential a, const nip_potential b) {
  if (a->dimensionality != b->dimensionality) return false;
  for (int i = 0; i < a->dimensionality; i++)
    if (a->cardinality[i] != b->cardinality[i]) return false;
  return true;
}

}  // namespace

extern "C" {

nip_potential nip_new_potential(int cardinality[], int dimensionality, double data[]) {
  if (dimensionality < 0) {
    REPORT(EINVAL);
    return nullptr;
  }
  auto* p = (nip_potential)std::calloc(1, sizeof(nip_potential_struct));
  if (!p) {
    REPORT(ENOMEM);
    return nullptr;
  }
  const int nd = dimensionality > 0 ? dimensionality : 1;
  p->cardinality = (int*)std::calloc(nd, sizeof(int));
  p->temp_index = (int*)std::calloc(nd, sizeof(int));
  if (!p->cardinality || !p->temp_index) {
    REPORT(ENOMEM);
    nip_free_potential(p);
    return nullptr;
  }
  p->dimensionality = dimensionality;
  int size = 1;
  for (int i = 0; i < dimensionality; i++) {
    p->cardinality[i] = cardinality[i];
    size *= cardinality[i];
  }
  if (dimensionality == 0) p->cardinality[0] = 1;  // a scalar weight (:126-128)
  p->size_of_data = size;
  p->data = (double*)std::malloc(sizeof(double) * (size > 0 ? size : 1));
  if (!p->data) {
    REPORT(ENOMEM);
    nip_free_potential(p);
    return nullptr;
  }
  if (data) {
    std::memcpy(p->data, data, sizeof(double) * size);
  } else {
    for (int i = 0; i < size; i++) p->data[i] = 1.0;
  }
  p->application_specific_properties = nip_new_string_pair_list();
  return p;
}

int nip_set_potential_property(nip_potential p, char* key, char* value) {
  if (!p || !key || !value) return REPORT(EFAULT);
  return nip_append_string_pair(p->application_specific_properties, key, value);
}

char* nip_get_potential_property(nip_potential p, char* key) {
  if (!p || !key) {
    REPORT(EFAULT);
    return nullptr;
  }
  return nip_string_pair_list_search(p->application_specific_properties, key);
}

nip_potential nip_copy_potential(nip_potential p) {
  if (!p) return nullptr;
  return nip_new_potential(p->cardinality, p->dimensionality, p->data);  // properties not copied (:178)
}

int nip_retract_potential(nip_potential p, nip_potential ref) {
  if (!p || !ref) return REPORT(EFAULT);
  if (!same_geometry(p, ref)) return REPORT(EINVAL);
  std::memcpy(p->data, ref->data, sizeof(double) * p->size_of_data);
  return 0;
}

void nip_free_potential(nip_potential p) {
  if (!p) return;
  nip_free_string_pair_list(p->application_specific_properties);
  std::free(p->cardinality);
  std::free(p->temp_index);
  std::free(p->data);
  std::free(p);
}

void nip_uniform_potential(nip_potential p, double value) {
  if (!p) return;
  for (int i = 0; i < p->size_of_data; i++) p->data[i] = value;
}

// draws from the caller's rand() stream, one per entry (:222-230)
void nip_random_potential(nip_potential p) {
  if (!p) return;
  for (int i = 0; i < p->size_of_data; i++) p->data[i] = std::rand() / (double)RAND_MAX;
}

namespace {
long flat_of(const nip_potential p, const int* indices) {
  long f = 0, s = 1;
  for (int i = 0; i < p->dimensionality; i++) {
    f += (long)indices[i] * s;
    s *= p->cardinality[i];
  }
  return f;
}
}  // namespace

double nip_get_potential_value(nip_potential p, int indices[]) { return p->data[flat_of(p, indices)]; }

void nip_set_potential_value(nip_potential p, int indices[], double value) {
  p->data[flat_of(p, indices)] = value;
}

void nip_inverse_mapping(nip_potential p, int flat_index, int indices[]) {
  for (int i = 0; i < p->dimensionality; i++) {
    indices[i] = flat_index % p->cardinality[i];
    flat_index /= p->cardinality[i];
  }
}

int nip_general_marginalise(nip_potential source, nip_potential destination, int mapping[]) {
  if (destination->dimensionality > source->dimensionality) return REPORT(EINVAL);
  if (destination->dimensionality == 0) {
    double s = 0.0;
    for (int i = 0; i < source->size_of_data; i++) s += source->data[i];
    destination->data[0] = s;
    return 0;
  }
  double* d = destination->data;
  const double* x = source->data;
  for (int j = 0; j < destination->size_of_data; j++) d[j] = 0.0;
  walk_projection(source, mapping, destination->dimensionality, destination->cardinality,
                  [&](int i, long j) { d[j] += x[i]; });
  return 0;
}

int nip_total_marginalise(nip_potential source, double destination[], int variable) {
  if (variable < 0 || variable >= source->dimensionality) return REPORT(EINVAL);
  const int card = source->cardinality[variable];
  for (int k = 0; k < card; k++) destination[k] = 0.0;
  const int map[1] = {variable};
  walk_projection(source, map, 1, &card, [&](int i, long k) { destination[k] += source->data[i]; });
  return 0;
}

void nip_normalise_array(double result[], int array_size) {
  double sum = 0.0;
  for (int i = 0; i < array_size; i++) sum += result[i];
  if (sum == 0.0) return;
  for (int i = 0; i < array_size; i++) result[i] /= sum;
}

int nip_normalise_potential(nip_potential p) {
  if (!p) return REPORT(EFAULT);
  nip_normalise_array(p->data, p->size_of_data);
  return 0;
}

// every run of card[0] consecutive entries is one distribution of the
// dimension-0 variable (:373-383)
int nip_normalise_cpd(nip_potential p) {
  if (!p) return REPORT(EFAULT);
  const int n = p->cardinality[0];
  for (int i = 0; i < p->size_of_data; i += n) nip_normalise_array(p->data + i, n);
  return 0;
}

// marginalise onto every other dimension, then divide (0 where that sum is
// 0), as the reference's general_marginalise + update_potential pair (:387-418)
int nip_normalise_dimension(nip_potential p, int dimension) {
  if (!p || dimension < 0 || dimension >= p->dimensionality) return REPORT(EINVAL);
  std::vector<int> card, map;
  for (int i = 0; i < p->dimensionality; i++)
    if (i != dimension) {
      card.push_back(p->cardinality[i]);
      map.push_back(i);
    }
  nip_potential den = nip_new_potential(card.data(), (int)card.size(), nullptr);
  if (!den) return REPORT(ENOMEM);
  nip_general_marginalise(p, den, map.data());
  nip_update_potential(nullptr, den, p, map.data());
  nip_free_potential(den);
  return 0;
}

int nip_sum_potential(nip_potential sum, nip_potential increment) {
  if (!sum || !increment || sum->size_of_data != increment->size_of_data) return REPORT(EFAULT);
  for (int i = 0; i < sum->size_of_data; i++) sum->data[i] += increment->data[i];
  return 0;
}

int nip_update_potential(nip_potential numerator, nip_potential denominator, nip_potential target,
                         int mapping[]) {
  if ((numerator && denominator && numerator->dimensionality != denominator->dimensionality) ||
      (!numerator && !denominator))
    return REPORT(EFAULT);
  const nip_potential g = numerator ? numerator : denominator;   // the sepset geometry
  const double* num = numerator ? numerator->data : nullptr;
  const double* den = denominator ? denominator->data : nullptr;
  double* t = target->data;
  auto apply = [&](int i, long j) {
    if (num) t[i] *= num[j];
    if (den) t[i] = den[j] != 0.0 ? t[i] / den[j] : 0.0;   // Procedural Guide p. 20
  };
  if (g->dimensionality == 0) {
    for (int i = 0; i < target->size_of_data; i++) apply(i, 0);
    return 0;
  }
  walk_projection(target, mapping, g->dimensionality, g->cardinality, apply);
  return 0;
}

int nip_update_evidence(double numerator[], double denominator[], nip_potential target, int var) {
  const int card = target->cardinality[var];
  const int map[1] = {var};
  double* t = target->data;
  walk_projection(target, map, 1, &card, [&](int i, long k) {
    t[i] *= numerator[k];
    if (denominator && denominator[k] != 0.0) t[i] /= denominator[k];
  });
  return 0;
}

int nip_init_potential(nip_potential probs, nip_potential target, int mapping[]) {
  if (!mapping) {
    if (probs->size_of_data != target->size_of_data) return REPORT(EFAULT);
    for (int i = 0; i < target->size_of_data; i++) target->data[i] *= probs->data[i];
    return 0;
  }
  if (probs->dimensionality == 0) return 0;
  double* t = target->data;
  const double* q = probs->data;
  walk_projection(target, mapping, probs->dimensionality, probs->cardinality,
                  [&](int i, long j) { t[i] *= q[j]; });
  return 0;
}

void nip_fprintf_potential(FILE* stream, nip_potential p) {
  if (p->dimensionality == 0) {
    std::fprintf(stream, "P(0) = %f\n", p->data[0]);
    return;
  }
  std::vector<int> idx(p->dimensionality);
  for (int i = 0; i < p->size_of_data; i++) {
    nip_inverse_mapping(p, i, idx.data());
    std::fprintf(stream, "P(");
    for (int k = 0; k < p->dimensionality; k++)
      std::fprintf(stream, k + 1 < p->dimensionality ? "%d, " : "%d", idx[k]);
    std::fprintf(stream, ") = %f\n", p->data[i]);
  }
}

}  // extern "C"
