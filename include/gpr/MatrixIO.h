// gpr/MatrixIO.h — the reference's binary matrix file format (lib/MatrixIO.cpp:38-100):
// an ASCII header "rows cols\n" followed by the raw row-major payload in the scalar type.
// Files written by the reference load here and vice versa.
#pragma once

#include <fstream>
#include <sstream>
#include <string>
#include <vector>

#include "Matrix.h"

namespace gpr {

template <class M>
M ReadMatrix(const std::string& filename) {
    typedef typename M::Scalar S;
    std::ifstream in(filename.c_str(), std::ios::binary);
    std::string line;
    unsigned long long rows = 0, cols = 0;
    if (!in || !std::getline(in, line)) {
        std::stringstream e;
        e << "ReadMatrix: header is corrupt (filename " << filename << ")." << std::endl;
        throw e.str();
    }
    std::istringstream hs(line);
    if (!(hs >> rows && hs >> cols)) {
        std::stringstream e;
        e << "ReadMatrix: header is corrupt (filename " << filename << ")." << std::endl;
        throw e.str();
    }
    M m(rows, cols);
    in.read(reinterpret_cast<char*>(m.data()), (std::streamsize)(rows * cols * sizeof(S)));
    return m;
}

template <class M>
void WriteMatrix(const M& m, const std::string& filename) {
    typedef typename M::Scalar S;
    std::ofstream out(filename.c_str(), std::ios::binary);
    std::ostringstream hs;
    hs << (unsigned long long)m.rows() << " " << (unsigned long long)m.cols() << std::endl;
    const std::string h = hs.str();
    out.write(h.data(), (std::streamsize)h.size());
    out.write(reinterpret_cast<const char*>(m.data()), (std::streamsize)(m.rows() * m.cols() * sizeof(S)));
}

}  // namespace gpr
