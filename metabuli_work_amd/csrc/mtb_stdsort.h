// Exact emulation of libstdc++'s std::sort (introsort: median-of-3 pivot moved to first,
// unguarded Hoare partition, depth limit 2*floor(log2 n) falling back to heapsort, final
// insertion sort with threshold 16) as a host/device template.
//
// Why: Taxonomer::combineMatchPaths (Taxonomer.cpp:417-426) sorts MatchPaths with a comparator
// that is not a total order (paths can tie on score, hamming and start while differing in end),
// so the order of tied paths — and through the greedy overlap trimming, the species score — is
// whatever the reference's std::sort produces. The reference is built with GCC/libstdc++; this
// reproduces that algorithm step for step so the device result is bit-identical.
// tests/test_stdsort.py checks it against the host libstdc++ std::sort on adversarial inputs.
#pragma once

#if defined(__HIPCC__)
#define MTB_HD __host__ __device__
#else
#define MTB_HD
#endif

namespace mtb {
namespace stdsort {

template <typename T>
MTB_HD inline void swap_(T& a, T& b) {
    T t = a;
    a = b;
    b = t;
}

MTB_HD inline long lg(long n) {  // std::__lg
    long k = 0;
    while ((n >> (k + 1)) > 0) k++;
    return k;
}

template <typename T, typename C>
MTB_HD inline void move_median_to_first(T* result, T* a, T* b, T* c, C comp) {
    if (comp(*a, *b)) {
        if (comp(*b, *c)) swap_(*result, *b);
        else if (comp(*a, *c)) swap_(*result, *c);
        else swap_(*result, *a);
    } else if (comp(*a, *c)) swap_(*result, *a);
    else if (comp(*b, *c)) swap_(*result, *c);
    else swap_(*result, *b);
}

template <typename T, typename C>
MTB_HD inline T* unguarded_partition(T* first, T* last, T* pivot, C comp) {
    while (true) {
        while (comp(*first, *pivot)) ++first;
        --last;
        while (comp(*pivot, *last)) --last;
        if (!(first < last)) return first;
        swap_(*first, *last);
        ++first;
    }
}

template <typename T, typename C>
MTB_HD inline void push_heap_(T* first, long hole, long top, T value, C comp) {
    long parent = (hole - 1) / 2;
    while (hole > top && comp(first[parent], value)) {
        first[hole] = first[parent];
        hole = parent;
        parent = (hole - 1) / 2;
    }
    first[hole] = value;
}

template <typename T, typename C>
MTB_HD inline void adjust_heap(T* first, long hole, long len, T value, C comp) {
    const long top = hole;
    long child = hole;
    while (child < (len - 1) / 2) {
        child = 2 * (child + 1);
        if (comp(first[child], first[child - 1])) child--;
        first[hole] = first[child];
        hole = child;
    }
    if ((len & 1) == 0 && child == (len - 2) / 2) {
        child = 2 * (child + 1);
        first[hole] = first[child - 1];
        hole = child - 1;
    }
    push_heap_(first, hole, top, value, comp);
}

template <typename T, typename C>
MTB_HD inline void make_heap_(T* first, T* last, C comp) {
    long len = last - first;
    if (len < 2) return;
    long parent = (len - 2) / 2;
    while (true) {
        T value = first[parent];
        adjust_heap(first, parent, len, value, comp);
        if (parent == 0) return;
        parent--;
    }
}

template <typename T, typename C>
MTB_HD inline void heap_sort_(T* first, T* last, C comp) {  // __partial_sort(first, last, last)
    make_heap_(first, last, comp);
    while (last - first > 1) {
        --last;
        T value = *last;
        *last = *first;
        adjust_heap(first, 0L, (long)(last - first), value, comp);
    }
}

template <typename T, typename C>
MTB_HD inline void unguarded_linear_insert(T* last, C comp) {
    T val = *last;
    T* next = last - 1;
    while (comp(val, *next)) {
        *last = *next;
        last = next;
        --next;
    }
    *last = val;
}

template <typename T, typename C>
MTB_HD inline void insertion_sort(T* first, T* last, C comp) {
    if (first == last) return;
    for (T* i = first + 1; i != last; ++i) {
        if (comp(*i, *first)) {
            T val = *i;
            for (T* p = i; p != first; --p) *p = *(p - 1);  // move_backward
            *first = val;
        } else {
            unguarded_linear_insert(i, comp);
        }
    }
}

template <typename T, typename C>
MTB_HD inline void introsort_loop(T* first, T* last, long depth, C comp) {
    // The reference recurses on the right part; an explicit stack of (cut, last, depth) keeps
    // the same visiting order without device recursion.
    struct Frame { T* f; T* l; long d; };
    Frame stack[64];
    int sp = 0;
    stack[sp++] = {first, last, depth};
    while (sp > 0) {
        Frame fr = stack[--sp];
        T* f = fr.f;
        T* l = fr.l;
        long d = fr.d;
        while (l - f > 16) {
            if (d == 0) {
                heap_sort_(f, l, comp);
                break;
            }
            --d;
            T* mid = f + (l - f) / 2;
            move_median_to_first(f, f + 1, mid, l - 1, comp);
            T* cut = unguarded_partition(f + 1, l, f, comp);
            // std::__introsort_loop(cut, last, depth) runs to completion before the loop
            // continues on [first, cut): process the right part first.
            stack[sp++] = {f, cut, d};
            f = cut;
            // continue with right part in this loop; the left part is resumed from the stack
            // after the right part finishes (LIFO order preserves the reference's sequencing).
            continue;
        }
    }
}

template <typename T, typename C>
MTB_HD inline void sort(T* first, T* last, C comp) {
    if (first == last) return;
    introsort_loop(first, last, lg((long)(last - first)) * 2, comp);
    if (last - first > 16) {  // __final_insertion_sort
        insertion_sort(first, first + 16, comp);
        for (T* i = first + 16; i != last; ++i) unguarded_linear_insert(i, comp);
    } else {
        insertion_sort(first, last, comp);
    }
}

}  // namespace stdsort
}  // namespace mtb
