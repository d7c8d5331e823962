// arma_lite.hpp -- the subset of Armadillo's dense types the PSO / costfunc / handmodel
// boundary uses (the reference passes arma::vec / mat / uvec by reference everywhere:
// PSO.h:56-68, costfunc.h:25-41, handmodel.h:9-32).  Used only when <armadillo> is not
// available (it is absent from this image); hpe_facade.hpp picks the real library
// otherwise.  Column-major storage with a contiguous memptr(), like Armadillo, so a
// 26 x P particle matrix hands over to the C ABI without a copy.
#pragma once
#include <cstddef>
#include <cstdint>
#include <initializer_list>
#include <stdexcept>
#include <vector>

namespace arma {

typedef unsigned long long uword;  // ARMA_64BIT_WORD (default for C++11 builds)

struct endr_marker {};
static const endr_marker endr = {};

template <typename eT>
class Mat {
public:
    typedef eT elem_type;
    uword n_rows = 0, n_cols = 0, n_elem = 0;

    Mat() = default;
    Mat(uword r, uword c) { set_size(r, c); }
    virtual ~Mat() = default;

    void set_size(uword r, uword c) {
        n_rows = r;
        n_cols = c;
        n_elem = r * c;
        mem_.assign((size_t)n_elem, eT(0));
        fill_pos_ = 0;
    }
    Mat &zeros(uword r, uword c) {
        set_size(r, c);
        return *this;
    }
    Mat &zeros() {
        for (auto &x : mem_) x = eT(0);
        return *this;
    }
    Mat &fill(eT v) {
        for (auto &x : mem_) x = v;
        return *this;
    }
    eT *memptr() { return mem_.data(); }
    const eT *memptr() const { return mem_.data(); }
    eT &operator()(uword i) { return at_checked(i); }
    const eT &operator()(uword i) const { return const_cast<Mat *>(this)->at_checked(i); }
    eT &operator()(uword r, uword c) { return at_checked(r + n_rows * c); }
    const eT &operator()(uword r, uword c) const {
        return const_cast<Mat *>(this)->at_checked(r + n_rows * c);
    }
    eT &at(uword r, uword c) { return mem_[(size_t)(r + n_rows * c)]; }
    const eT &at(uword r, uword c) const { return mem_[(size_t)(r + n_rows * c)]; }
    // Armadillo's "x0 << 1 << 2 << endr" element insertion (column-major order for vectors)
    Mat &operator<<(eT v) {
        at_checked(fill_pos_++) = v;
        return *this;
    }
    Mat &operator<<(endr_marker) { return *this; }

protected:
    eT &at_checked(uword i) {
        if (i >= n_elem) throw std::out_of_range("arma_lite: index out of bounds");
        return mem_[(size_t)i];
    }
    std::vector<eT> mem_;
    uword fill_pos_ = 0;
};

template <typename eT>
class Col : public Mat<eT> {
public:
    Col() { Mat<eT>::set_size(0, 1); }
    explicit Col(uword n) { Mat<eT>::set_size(n, 1); }
    Col(std::initializer_list<eT> l) {
        Mat<eT>::set_size(l.size(), 1);
        uword i = 0;
        for (const eT &v : l) this->mem_[(size_t)i++] = v;
    }
    void set_size(uword n) { Mat<eT>::set_size(n, 1); }
    void set_size(uword r, uword c) { Mat<eT>::set_size(r, c); }
    Col &zeros(uword n) {
        set_size(n);
        return *this;
    }
    Col &zeros() {
        Mat<eT>::zeros();
        return *this;
    }
};

typedef Mat<double> mat;
typedef Mat<float> fmat;
typedef Col<double> vec;
typedef Col<double> colvec;
typedef Col<uword> uvec;

template <typename T>
inline T zeros(uword n) {
    T v;
    v.zeros(n);
    return v;
}
template <typename T>
inline T zeros(uword r, uword c) {
    T m;
    m.zeros(r, c);
    return m;
}

}  // namespace arma
