// svd3.h -- 3x3 SVD in fp64 for the weighted-SVD pose head (layers.py:456-504):
// Jacobi eigen-decomposition of H^T H (right singular vectors, sigma^2), left
// vectors u_i = H v_i / |H v_i| (completed by cross products when H is rank
// deficient).  Shared by the forward (heads.hip) and its backward (train_ops.hip).
#pragma once
#include <hip/hip_runtime.h>

__device__ inline void jacobi3(double A[3][3], double V[3][3]) {
    for (int i = 0; i < 3; ++i)
        for (int j = 0; j < 3; ++j) V[i][j] = i == j ? 1.0 : 0.0;
    for (int sweep = 0; sweep < 50; ++sweep) {
        const double off = fabs(A[0][1]) + fabs(A[0][2]) + fabs(A[1][2]);
        const double dg = fabs(A[0][0]) + fabs(A[1][1]) + fabs(A[2][2]);
        if (off <= 1e-300 || off <= 1e-17 * dg) break;
        for (int p = 0; p < 2; ++p)
            for (int q = p + 1; q < 3; ++q) {
                if (A[p][q] == 0.0) continue;
                const double theta = (A[q][q] - A[p][p]) / (2.0 * A[p][q]);
                const double t = (theta >= 0 ? 1.0 : -1.0) / (fabs(theta) + sqrt(theta * theta + 1.0));
                const double c = 1.0 / sqrt(t * t + 1.0), s = t * c;
                for (int r = 0; r < 3; ++r) {  // A <- A J
                    const double arp = A[r][p], arq = A[r][q];
                    A[r][p] = c * arp - s * arq;
                    A[r][q] = s * arp + c * arq;
                }
                for (int r = 0; r < 3; ++r) {  // A <- J^T A
                    const double apr = A[p][r], aqr = A[q][r];
                    A[p][r] = c * apr - s * aqr;
                    A[q][r] = s * apr + c * aqr;
                }
                for (int r = 0; r < 3; ++r) {  // V <- V J
                    const double vrp = V[r][p], vrq = V[r][q];
                    V[r][p] = c * vrp - s * vrq;
                    V[r][q] = s * vrp + c * vrq;
                }
            }
    }
}

__device__ inline void cross3(const double a[3], const double b[3], double o[3]) {
    o[0] = a[1] * b[2] - a[2] * b[1];
    o[1] = a[2] * b[0] - a[0] * b[2];
    o[2] = a[0] * b[1] - a[1] * b[0];
}

// u[i], v[i]: i-th left / right singular vector (descending sig); returns det(V U^T) sign
__device__ inline double svd3_usv(const double H[3][3], double u[3][3], double sig[3],
                                  double v[3][3]) {

    double A[3][3], V[3][3];
    for (int i = 0; i < 3; ++i)
        for (int j = 0; j < 3; ++j) {
            double s = 0;
            for (int r = 0; r < 3; ++r) s += H[r][i] * H[r][j];
            A[i][j] = s;
        }
    jacobi3(A, V);
    double lam[3] = {A[0][0], A[1][1], A[2][2]};
    int ord[3] = {0, 1, 2};
    for (int i = 0; i < 3; ++i)
        for (int j = i + 1; j < 3; ++j)
            if (lam[ord[j]] > lam[ord[i]]) { const int t = ord[i]; ord[i] = ord[j]; ord[j] = t; }
    for (int i = 0; i < 3; ++i) {
        sig[i] = sqrt(fmax(lam[ord[i]], 0.0));
        for (int r = 0; r < 3; ++r) v[i][r] = V[r][ord[i]];
    }
    const double tiny = 1e-12 * (sig[0] > 0 ? sig[0] : 1.0);
    for (int i = 0; i < 3; ++i) {
        double hv[3];
        for (int r = 0; r < 3; ++r) hv[r] = H[r][0] * v[i][0] + H[r][1] * v[i][1] + H[r][2] * v[i][2];
        const double nrm = sqrt(hv[0] * hv[0] + hv[1] * hv[1] + hv[2] * hv[2]);
        if (sig[i] > tiny && nrm > 0) {
            for (int r = 0; r < 3; ++r) u[i][r] = hv[r] / nrm;
        } else if (i == 2) {
            cross3(u[0], u[1], u[2]);
        } else if (i == 1) {
            // any unit vector orthogonal to u0
            const double e[3] = {fabs(u[0][0]) < 0.9 ? 1.0 : 0.0, fabs(u[0][0]) < 0.9 ? 0.0 : 1.0, 0.0};
            double c[3];
            cross3(u[0], e, c);
            const double cn = sqrt(c[0] * c[0] + c[1] * c[1] + c[2] * c[2]);
            for (int r = 0; r < 3; ++r) u[1][r] = c[r] / cn;
        } else {
            for (int r = 0; r < 3; ++r) u[0][r] = r == 0 ? 1.0 : 0.0;
        }
    }
    // det(V U^T) = det(V) det(U)
    double c01[3];
    cross3(v[0], v[1], c01);
    const double dv = c01[0] * v[2][0] + c01[1] * v[2][1] + c01[2] * v[2][2];
    cross3(u[0], u[1], c01);
    const double du = c01[0] * u[2][0] + c01[1] * u[2][1] + c01[2] * u[2][2];
    const double d = dv * du < 0 ? -1.0 : 1.0;
    return d;
}
