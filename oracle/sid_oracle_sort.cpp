// oracle/sid_oracle_sort.cpp -- TEST INFRASTRUCTURE ONLY (part of the oracle).
// stats.cpp:58-66 descending_sorted_indices: std::sort over the indices with
// the reference's comparator v[i] > v[j].  With NaN p-values (a profile whose
// long double likelihood is 0 * inf) that comparator is no strict weak order,
// and where the NaNs land -- which moves every later adjusted p-value of
// adjustBenjaminiHochberg -- is what libstdc++'s introsort does with it; a
// qsort with an index tie-break puts them elsewhere.  Same template, same
// comparator, same input order as the reference.
#include <algorithm>
#include <cstddef>

extern "C" void oracle_descending_sorted_indices(const double* v, size_t m, size_t* idx)
{
    for (size_t i = 0; i < m; ++i) idx[i] = i;
    std::sort(idx, idx + m, [v](size_t i, size_t j) { return v[i] > v[j]; });
}
