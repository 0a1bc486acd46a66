// gpr/Matrix.h — minimal dense containers for the host API.
//
// The reference exposes Eigen types in its public signatures
// (include/GaussianProcess.h:41-46: VectorType = Eigen::Matrix<T,Dynamic,1>, MatrixType =
// Eigen::Matrix<T,Dynamic,Dynamic,RowMajor>).  Eigen is not part of this build, so the host
// layer ships these small row-major containers under the same typedef names with the
// subset of the Eigen interface the reference's callers use (construction by size,
// operator(), operator[], Zero/Random/Constant, rows/cols/size, resize, norm, col, data,
// element-wise + and -, scalar *, transpose, matrix * vector / matrix).
#pragma once

#include <cmath>
#include <cstddef>
#include <cstdlib>
#include <initializer_list>
#include <random>
#include <stdexcept>
#include <vector>

namespace gpr {

template <class T>
class DenseMatrix;

template <class T>
class DenseVector {
public:
    typedef T Scalar;
    DenseVector() {}
    explicit DenseVector(std::size_t n) : m_data(n, T(0)) {}
    DenseVector(std::initializer_list<T> v) : m_data(v) {}

    static DenseVector Zero(std::size_t n) { return DenseVector(n); }
    static DenseVector Constant(std::size_t n, T v) {
        DenseVector r(n);
        for (auto& x : r.m_data) x = v;
        return r;
    }
    // uniform in [-1, 1) like Eigen::Random
    static DenseVector Random(std::size_t n) {
        DenseVector r(n);
        for (auto& x : r.m_data) x = T(2) * T(std::rand()) / T(RAND_MAX) - T(1);
        return r;
    }

    std::size_t size() const { return m_data.size(); }
    std::size_t rows() const { return m_data.size(); }
    std::size_t cols() const { return 1; }
    void resize(std::size_t n) { m_data.assign(n, T(0)); }
    T& operator()(std::size_t i) { return m_data[i]; }
    const T& operator()(std::size_t i) const { return m_data[i]; }
    T& operator[](std::size_t i) { return m_data[i]; }
    const T& operator[](std::size_t i) const { return m_data[i]; }
    T* data() { return m_data.data(); }
    const T* data() const { return m_data.data(); }

    T squaredNorm() const {
        T s = 0;
        for (T x : m_data) s += x * x;
        return s;
    }
    T norm() const { return std::sqrt(squaredNorm()); }
    T sum() const {
        T s = 0;
        for (T x : m_data) s += x;
        return s;
    }
    DenseVector operator-(const DenseVector& b) const {
        check(b);
        DenseVector r(size());
        for (std::size_t i = 0; i < size(); i++) r[i] = m_data[i] - b[i];
        return r;
    }
    DenseVector operator+(const DenseVector& b) const {
        check(b);
        DenseVector r(size());
        for (std::size_t i = 0; i < size(); i++) r[i] = m_data[i] + b[i];
        return r;
    }
    DenseVector operator*(T s) const {
        DenseVector r(*this);
        for (auto& x : r.m_data) x *= s;
        return r;
    }
    DenseVector& operator+=(const DenseVector& b) {
        check(b);
        for (std::size_t i = 0; i < size(); i++) m_data[i] += b[i];
        return *this;
    }
    bool operator==(const DenseVector& b) const { return m_data == b.m_data; }

private:
    void check(const DenseVector& b) const {
        if (b.size() != size()) throw std::string("DenseVector: size mismatch");
    }
    std::vector<T> m_data;
};

template <class T>
class DenseMatrix {
public:
    typedef T Scalar;
    DenseMatrix() : m_rows(0), m_cols(0) {}
    DenseMatrix(std::size_t r, std::size_t c) : m_rows(r), m_cols(c), m_data(r * c, T(0)) {}

    static DenseMatrix Zero(std::size_t r, std::size_t c) { return DenseMatrix(r, c); }
    static DenseMatrix Identity(std::size_t r, std::size_t c) {
        DenseMatrix m(r, c);
        for (std::size_t i = 0; i < r && i < c; i++) m(i, i) = T(1);
        return m;
    }
    static DenseMatrix Random(std::size_t r, std::size_t c) {
        DenseMatrix m(r, c);
        for (auto& x : m.m_data) x = T(2) * T(std::rand()) / T(RAND_MAX) - T(1);
        return m;
    }

    std::size_t rows() const { return m_rows; }
    std::size_t cols() const { return m_cols; }
    std::size_t size() const { return m_data.size(); }
    // Eigen's diagonalSize(): min(rows, cols) (used by the reference's lazy core-matrix test)
    std::size_t diagonalSize() const { return m_rows < m_cols ? m_rows : m_cols; }
    void resize(std::size_t r, std::size_t c) {
        m_rows = r;
        m_cols = c;
        m_data.assign(r * c, T(0));
    }
    void setZero(std::size_t r, std::size_t c) { resize(r, c); }
    T& operator()(std::size_t i, std::size_t j) { return m_data[i * m_cols + j]; }
    const T& operator()(std::size_t i, std::size_t j) const { return m_data[i * m_cols + j]; }
    T* data() { return m_data.data(); }
    const T* data() const { return m_data.data(); }

    DenseVector<T> col(std::size_t j) const {
        DenseVector<T> v(m_rows);
        for (std::size_t i = 0; i < m_rows; i++) v[i] = (*this)(i, j);
        return v;
    }
    DenseVector<T> row(std::size_t i) const {
        DenseVector<T> v(m_cols);
        for (std::size_t j = 0; j < m_cols; j++) v[j] = (*this)(i, j);
        return v;
    }
    void setCol(std::size_t j, const DenseVector<T>& v) {
        for (std::size_t i = 0; i < m_rows; i++) (*this)(i, j) = v[i];
    }
    DenseMatrix transpose() const {
        DenseMatrix t(m_cols, m_rows);
        for (std::size_t i = 0; i < m_rows; i++)
            for (std::size_t j = 0; j < m_cols; j++) t(j, i) = (*this)(i, j);
        return t;
    }
    DenseMatrix operator-(const DenseMatrix& b) const {
        same(b);
        DenseMatrix r(m_rows, m_cols);
        for (std::size_t e = 0; e < m_data.size(); e++) r.m_data[e] = m_data[e] - b.m_data[e];
        return r;
    }
    DenseMatrix operator+(const DenseMatrix& b) const {
        same(b);
        DenseMatrix r(m_rows, m_cols);
        for (std::size_t e = 0; e < m_data.size(); e++) r.m_data[e] = m_data[e] + b.m_data[e];
        return r;
    }
    DenseVector<T> operator*(const DenseVector<T>& v) const {
        if (v.size() != m_cols) throw std::string("DenseMatrix: size mismatch in matrix * vector");
        DenseVector<T> r(m_rows);
        for (std::size_t i = 0; i < m_rows; i++) {
            T s = 0;
            for (std::size_t j = 0; j < m_cols; j++) s += (*this)(i, j) * v[j];
            r[i] = s;
        }
        return r;
    }
    DenseMatrix operator*(const DenseMatrix& b) const {
        if (b.m_rows != m_cols) throw std::string("DenseMatrix: size mismatch in matrix * matrix");
        DenseMatrix r(m_rows, b.m_cols);
        for (std::size_t i = 0; i < m_rows; i++)
            for (std::size_t k = 0; k < m_cols; k++) {
                const T a = (*this)(i, k);
                for (std::size_t j = 0; j < b.m_cols; j++) r(i, j) += a * b(k, j);
            }
        return r;
    }
    T squaredNorm() const {
        T s = 0;
        for (T x : m_data) s += x * x;
        return s;
    }
    T norm() const { return std::sqrt(squaredNorm()); }

private:
    void same(const DenseMatrix& b) const {
        if (b.m_rows != m_rows || b.m_cols != m_cols) throw std::string("DenseMatrix: size mismatch");
    }
    std::size_t m_rows, m_cols;
    std::vector<T> m_data;
};

}  // namespace gpr
