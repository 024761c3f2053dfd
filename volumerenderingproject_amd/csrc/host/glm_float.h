// glm_float.h -- the slice of glm 0.9.8.5 arithmetic the render path uses, with glm's exact
// float operation order (compiled with -ffp-contract=off), so host-side camera and TEST matrices
// match the reference bit for bit.  Column-major like glm::mat4 (m.c[col][row]).
//
// Op orders restated from the reference's vendored glm:
//   mat4*vec4  (m0*v0 + m1*v1) + (m2*v2 + m3*v3)          glm/detail/type_mat4x4.inl:526-537
//   mat4*mat4  ((A0*b0 + A1*b1) + A2*b2) + A3*b3 per column  type_mat4x4.inl:595-612
//   dot3       (x*x' + y*y') + z*z'                           glm/detail/func_geometric.inl:54-61
//   normalize  v * (1 / sqrt(dot(v, v)))                      func_geometric.inl:88-95
//   inverse    cofactor form                                  glm/detail/func_matrix.inl:297-354
//   lookAtRH / translate / scale / rotate                     glm/gtc/matrix_transform.inl
#pragma once
#include <cmath>

namespace vr {
namespace glmf {

struct vec3 { float x, y, z; };
struct vec4 { float x, y, z, w; };
struct mat4 { vec4 c[4]; };

inline vec3 v3(float x, float y, float z) { return {x, y, z}; }
inline vec4 v4(float x, float y, float z, float w) { return {x, y, z, w}; }
inline vec3 operator+(vec3 a, vec3 b) { return {a.x + b.x, a.y + b.y, a.z + b.z}; }
inline vec3 operator-(vec3 a, vec3 b) { return {a.x - b.x, a.y - b.y, a.z - b.z}; }
inline vec3 operator-(vec3 a) { return {-a.x, -a.y, -a.z}; }
inline vec3 operator*(float s, vec3 a) { return {s * a.x, s * a.y, s * a.z}; }
inline vec3 operator*(vec3 a, float s) { return {a.x * s, a.y * s, a.z * s}; }
inline vec4 operator+(vec4 a, vec4 b) { return {a.x + b.x, a.y + b.y, a.z + b.z, a.w + b.w}; }
inline vec4 operator-(vec4 a, vec4 b) { return {a.x - b.x, a.y - b.y, a.z - b.z, a.w - b.w}; }
inline vec4 operator*(vec4 a, vec4 b) { return {a.x * b.x, a.y * b.y, a.z * b.z, a.w * b.w}; }
inline vec4 operator*(vec4 a, float s) { return {a.x * s, a.y * s, a.z * s, a.w * s}; }
inline float at(const vec4& v, int i) { return i == 0 ? v.x : i == 1 ? v.y : i == 2 ? v.z : v.w; }

inline float dot(vec3 a, vec3 b) {
    vec3 t{a.x * b.x, a.y * b.y, a.z * b.z};
    return t.x + t.y + t.z;
}
inline vec3 cross(vec3 x, vec3 y) {
    return {x.y * y.z - y.y * x.z, x.z * y.x - y.z * x.x, x.x * y.y - y.x * x.y};
}
inline vec3 normalize(vec3 v) { return v * (1.0f / std::sqrt(dot(v, v))); }

inline mat4 identity() {
    return {{{1, 0, 0, 0}, {0, 1, 0, 0}, {0, 0, 1, 0}, {0, 0, 0, 1}}};
}
inline vec4 mul(const mat4& m, vec4 v) {
    vec4 add0 = m.c[0] * v.x + m.c[1] * v.y;
    vec4 add1 = m.c[2] * v.z + m.c[3] * v.w;
    return add0 + add1;
}
inline mat4 mul(const mat4& a, const mat4& b) {
    mat4 r;
    for (int j = 0; j < 4; ++j)
        r.c[j] = ((a.c[0] * b.c[j].x + a.c[1] * b.c[j].y) + a.c[2] * b.c[j].z) + a.c[3] * b.c[j].w;
    return r;
}
inline mat4 translate(const mat4& m, vec3 v) {
    mat4 r = m;
    r.c[3] = ((m.c[0] * v.x + m.c[1] * v.y) + m.c[2] * v.z) + m.c[3];
    return r;
}
inline mat4 scale(const mat4& m, vec3 v) {
    return {{m.c[0] * v.x, m.c[1] * v.y, m.c[2] * v.z, m.c[3]}};
}
inline mat4 rotate(const mat4& m, float angle, vec3 v) {
    const float c = std::cos(angle), s = std::sin(angle);
    vec3 axis = normalize(v);
    vec3 temp = (1.0f - c) * axis;
    float R[3][3];
    R[0][0] = c + temp.x * axis.x;
    R[0][1] = temp.x * axis.y + s * axis.z;
    R[0][2] = temp.x * axis.z - s * axis.y;
    R[1][0] = temp.y * axis.x - s * axis.z;
    R[1][1] = c + temp.y * axis.y;
    R[1][2] = temp.y * axis.z + s * axis.x;
    R[2][0] = temp.z * axis.x + s * axis.y;
    R[2][1] = temp.z * axis.y - s * axis.x;
    R[2][2] = c + temp.z * axis.z;
    mat4 r;
    for (int j = 0; j < 3; ++j) r.c[j] = (m.c[0] * R[j][0] + m.c[1] * R[j][1]) + m.c[2] * R[j][2];
    r.c[3] = m.c[3];
    return r;
}
inline mat4 lookAt(vec3 eye, vec3 center, vec3 up) {
    const vec3 f = normalize(center - eye);
    const vec3 s = normalize(cross(f, up));
    const vec3 u = cross(s, f);
    mat4 r = identity();
    r.c[0].x = s.x; r.c[1].x = s.y; r.c[2].x = s.z;
    r.c[0].y = u.x; r.c[1].y = u.y; r.c[2].y = u.z;
    r.c[0].z = -f.x; r.c[1].z = -f.y; r.c[2].z = -f.z;
    r.c[3].x = -dot(s, eye);
    r.c[3].y = -dot(u, eye);
    r.c[3].z = dot(f, eye);
    return r;
}
inline mat4 inverse(const mat4& M) {
    auto m = [&](int i, int j) { return at(M.c[i], j); };
    const float C00 = m(2, 2) * m(3, 3) - m(3, 2) * m(2, 3), C02 = m(1, 2) * m(3, 3) - m(3, 2) * m(1, 3);
    const float C03 = m(1, 2) * m(2, 3) - m(2, 2) * m(1, 3), C04 = m(2, 1) * m(3, 3) - m(3, 1) * m(2, 3);
    const float C06 = m(1, 1) * m(3, 3) - m(3, 1) * m(1, 3), C07 = m(1, 1) * m(2, 3) - m(2, 1) * m(1, 3);
    const float C08 = m(2, 1) * m(3, 2) - m(3, 1) * m(2, 2), C10 = m(1, 1) * m(3, 2) - m(3, 1) * m(1, 2);
    const float C11 = m(1, 1) * m(2, 2) - m(2, 1) * m(1, 2), C12 = m(2, 0) * m(3, 3) - m(3, 0) * m(2, 3);
    const float C14 = m(1, 0) * m(3, 3) - m(3, 0) * m(1, 3), C15 = m(1, 0) * m(2, 3) - m(2, 0) * m(1, 3);
    const float C16 = m(2, 0) * m(3, 2) - m(3, 0) * m(2, 2), C18 = m(1, 0) * m(3, 2) - m(3, 0) * m(1, 2);
    const float C19 = m(1, 0) * m(2, 2) - m(2, 0) * m(1, 2), C20 = m(2, 0) * m(3, 1) - m(3, 0) * m(2, 1);
    const float C22 = m(1, 0) * m(3, 1) - m(3, 0) * m(1, 1), C23 = m(1, 0) * m(2, 1) - m(2, 0) * m(1, 1);
    const vec4 F0{C00, C00, C02, C03}, F1{C04, C04, C06, C07}, F2{C08, C08, C10, C11};
    const vec4 F3{C12, C12, C14, C15}, F4{C16, C16, C18, C19}, F5{C20, C20, C22, C23};
    const vec4 V0{m(1, 0), m(0, 0), m(0, 0), m(0, 0)}, V1{m(1, 1), m(0, 1), m(0, 1), m(0, 1)};
    const vec4 V2{m(1, 2), m(0, 2), m(0, 2), m(0, 2)}, V3{m(1, 3), m(0, 3), m(0, 3), m(0, 3)};
    const vec4 I0 = (V1 * F0 - V2 * F1) + V3 * F2, I1 = (V0 * F0 - V2 * F3) + V3 * F4;
    const vec4 I2 = (V0 * F1 - V1 * F3) + V3 * F5, I3 = (V0 * F2 - V1 * F4) + V2 * F5;
    const vec4 SA{+1, -1, +1, -1}, SB{-1, +1, -1, +1};
    mat4 inv{{I0 * SA, I1 * SB, I2 * SA, I3 * SB}};
    const vec4 row0{inv.c[0].x, inv.c[1].x, inv.c[2].x, inv.c[3].x};
    const vec4 d0 = M.c[0] * row0;
    const float d1 = (d0.x + d0.y) + (d0.z + d0.w);
    const float od = 1.0f / d1;
    for (int i = 0; i < 4; ++i) inv.c[i] = inv.c[i] * od;
    return inv;
}

}  // namespace glmf
}  // namespace vr
