/*
 * vr_oracle.c -- CPU restatement of the reference volume-render hot path (TEST INFRASTRUCTURE).
 * See vr_oracle.h for the file:line map into /root/reference.  Build: oracle/Makefile
 * (gcc -O2 -ffp-contract=off, no fast-math: every float op rounds exactly as the reference's
 * scalar glm code does on an IEEE-754 single-precision machine).
 */
#include "vr_oracle.h"

#include <math.h>
#include <stdio.h>
#include <stdlib.h>
#include <string.h>
#ifdef _OPENMP
#include <omp.h>
#endif

/* =========================== glm 0.9.8.5 arithmetic, restated ========================= */

static inline or_v3 v3(float x, float y, float z) { or_v3 r = {x, y, z}; return r; }
static inline or_v4 v4(float x, float y, float z, float w) { or_v4 r = {x, y, z, w}; return r; }
static inline or_v3 v3_add(or_v3 a, or_v3 b) { return v3(a.x + b.x, a.y + b.y, a.z + b.z); }
static inline or_v3 v3_sub(or_v3 a, or_v3 b) { return v3(a.x - b.x, a.y - b.y, a.z - b.z); }
static inline or_v3 cam_v(const float* a) { return v3(a[0], a[1], a[2]); }
static inline or_v3 v3_neg(or_v3 a) { return v3(-a.x, -a.y, -a.z); }
static inline or_v3 sv3(float s, or_v3 a) { return v3(s * a.x, s * a.y, s * a.z); }    /* scalar*vec */
static inline or_v3 v3s(or_v3 a, float s) { return v3(a.x * s, a.y * s, a.z * s); }    /* vec*scalar */
static inline or_v4 v4_add(or_v4 a, or_v4 b) { return v4(a.x + b.x, a.y + b.y, a.z + b.z, a.w + b.w); }
static inline or_v4 v4_sub(or_v4 a, or_v4 b) { return v4(a.x - b.x, a.y - b.y, a.z - b.z, a.w - b.w); }
static inline or_v4 v4_mul(or_v4 a, or_v4 b) { return v4(a.x * b.x, a.y * b.y, a.z * b.z, a.w * b.w); }
static inline or_v4 v4s(or_v4 a, float s) { return v4(a.x * s, a.y * s, a.z * s, a.w * s); }
static inline float v4_get(or_v4 a, int i) { return i == 0 ? a.x : i == 1 ? a.y : i == 2 ? a.z : a.w; }
static inline void v4_set(or_v4* a, int i, float f) {
    if (i == 0) a->x = f; else if (i == 1) a->y = f; else if (i == 2) a->z = f; else a->w = f;
}

/* func_geometric.inl:54-61: tmp = x*y; return tmp.x + tmp.y + tmp.z */
static inline float v3_dot(or_v3 a, or_v3 b) {
    or_v3 t = v3(a.x * b.x, a.y * b.y, a.z * b.z);
    return t.x + t.y + t.z;
}
/* func_geometric.inl:74-85 */
or_v3 or_glm_cross(or_v3 x, or_v3 y) {
    return v3(x.y * y.z - y.y * x.z, x.z * y.x - y.z * x.x, x.x * y.y - y.x * x.y);
}
/* func_geometric.inl:88-95 + func_exponential.inl:128-133: v * (1 / sqrt(dot(v, v))) */
or_v3 or_glm_normalize(or_v3 v) {
    float inv = 1.0f / sqrtf(v3_dot(v, v));
    return v3s(v, inv);
}

static or_m4 m4_identity(void) {
    or_m4 m;
    m.c[0] = v4(1, 0, 0, 0); m.c[1] = v4(0, 1, 0, 0); m.c[2] = v4(0, 0, 1, 0); m.c[3] = v4(0, 0, 0, 1);
    return m;
}

/* type_mat4x4.inl:526-537: (m0*v0 + m1*v1) + (m2*v2 + m3*v3) */
or_v4 or_glm_mulv(or_m4 m, or_v4 v) {
    or_v4 add0 = v4_add(v4s(m.c[0], v.x), v4s(m.c[1], v.y));
    or_v4 add1 = v4_add(v4s(m.c[2], v.z), v4s(m.c[3], v.w));
    return v4_add(add0, add1);
}
/* type_mat4x4.inl:595-612: Result[j] = A0*B[j][0] + A1*B[j][1] + A2*B[j][2] + A3*B[j][3] */
or_m4 or_glm_mul(or_m4 a, or_m4 b) {
    or_m4 r;
    for (int j = 0; j < 4; ++j) {
        or_v4 acc = v4s(a.c[0], b.c[j].x);
        acc = v4_add(acc, v4s(a.c[1], b.c[j].y));
        acc = v4_add(acc, v4s(a.c[2], b.c[j].z));
        acc = v4_add(acc, v4s(a.c[3], b.c[j].w));
        r.c[j] = acc;
    }
    return r;
}
/* gtc/matrix_transform.inl:11-16: Result[3] = m0*v0 + m1*v1 + m2*v2 + m3 */
or_m4 or_glm_translate(or_m4 m, or_v3 v) {
    or_m4 r = m;
    or_v4 acc = v4s(m.c[0], v.x);
    acc = v4_add(acc, v4s(m.c[1], v.y));
    acc = v4_add(acc, v4s(m.c[2], v.z));
    r.c[3] = v4_add(acc, m.c[3]);
    return r;
}
/* gtc/matrix_transform.inl:79-87 */
or_m4 or_glm_scale(or_m4 m, or_v3 v) {
    or_m4 r;
    r.c[0] = v4s(m.c[0], v.x); r.c[1] = v4s(m.c[1], v.y); r.c[2] = v4s(m.c[2], v.z); r.c[3] = m.c[3];
    return r;
}
/* gtc/matrix_transform.inl:18-46 (angle in radians; cos/sin of float) */
or_m4 or_glm_rotate(or_m4 m, float angle, or_v3 v) {
    float c = cosf(angle), s = sinf(angle);
    or_v3 axis = or_glm_normalize(v);
    or_v3 temp = sv3(1.0f - c, axis);
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
    or_m4 r;
    for (int j = 0; j < 3; ++j) {
        or_v4 acc = v4s(m.c[0], R[j][0]);
        acc = v4_add(acc, v4s(m.c[1], R[j][1]));
        acc = v4_add(acc, v4s(m.c[2], R[j][2]));
        r.c[j] = acc;
    }
    r.c[3] = m.c[3];
    return r;
}
/* gtc/matrix_transform.inl:521-546 (lookAtRH, the default) */
or_m4 or_glm_lookat(or_v3 eye, or_v3 center, or_v3 up) {
    or_v3 f = or_glm_normalize(v3_sub(center, eye));
    or_v3 s = or_glm_normalize(or_glm_cross(f, up));
    or_v3 u = or_glm_cross(s, f);
    or_m4 r = m4_identity();
    r.c[0].x = s.x; r.c[1].x = s.y; r.c[2].x = s.z;
    r.c[0].y = u.x; r.c[1].y = u.y; r.c[2].y = u.z;
    r.c[0].z = -f.x; r.c[1].z = -f.y; r.c[2].z = -f.z;
    r.c[3].x = -v3_dot(s, eye);
    r.c[3].y = -v3_dot(u, eye);
    r.c[3].z = v3_dot(f, eye);
    return r;
}
/* detail/func_matrix.inl:297-354 */
or_m4 or_glm_inverse(or_m4 M) {
#define m(i, j) v4_get(M.c[i], j)
    float Coef00 = m(2,2) * m(3,3) - m(3,2) * m(2,3);
    float Coef02 = m(1,2) * m(3,3) - m(3,2) * m(1,3);
    float Coef03 = m(1,2) * m(2,3) - m(2,2) * m(1,3);
    float Coef04 = m(2,1) * m(3,3) - m(3,1) * m(2,3);
    float Coef06 = m(1,1) * m(3,3) - m(3,1) * m(1,3);
    float Coef07 = m(1,1) * m(2,3) - m(2,1) * m(1,3);
    float Coef08 = m(2,1) * m(3,2) - m(3,1) * m(2,2);
    float Coef10 = m(1,1) * m(3,2) - m(3,1) * m(1,2);
    float Coef11 = m(1,1) * m(2,2) - m(2,1) * m(1,2);
    float Coef12 = m(2,0) * m(3,3) - m(3,0) * m(2,3);
    float Coef14 = m(1,0) * m(3,3) - m(3,0) * m(1,3);
    float Coef15 = m(1,0) * m(2,3) - m(2,0) * m(1,3);
    float Coef16 = m(2,0) * m(3,2) - m(3,0) * m(2,2);
    float Coef18 = m(1,0) * m(3,2) - m(3,0) * m(1,2);
    float Coef19 = m(1,0) * m(2,2) - m(2,0) * m(1,2);
    float Coef20 = m(2,0) * m(3,1) - m(3,0) * m(2,1);
    float Coef22 = m(1,0) * m(3,1) - m(3,0) * m(1,1);
    float Coef23 = m(1,0) * m(2,1) - m(2,0) * m(1,1);
    or_v4 Fac0 = v4(Coef00, Coef00, Coef02, Coef03);
    or_v4 Fac1 = v4(Coef04, Coef04, Coef06, Coef07);
    or_v4 Fac2 = v4(Coef08, Coef08, Coef10, Coef11);
    or_v4 Fac3 = v4(Coef12, Coef12, Coef14, Coef15);
    or_v4 Fac4 = v4(Coef16, Coef16, Coef18, Coef19);
    or_v4 Fac5 = v4(Coef20, Coef20, Coef22, Coef23);
    or_v4 Vec0 = v4(m(1,0), m(0,0), m(0,0), m(0,0));
    or_v4 Vec1 = v4(m(1,1), m(0,1), m(0,1), m(0,1));
    or_v4 Vec2 = v4(m(1,2), m(0,2), m(0,2), m(0,2));
    or_v4 Vec3 = v4(m(1,3), m(0,3), m(0,3), m(0,3));
    /* a - b + c is (a - b) + c */
    or_v4 Inv0 = v4_add(v4_sub(v4_mul(Vec1, Fac0), v4_mul(Vec2, Fac1)), v4_mul(Vec3, Fac2));
    or_v4 Inv1 = v4_add(v4_sub(v4_mul(Vec0, Fac0), v4_mul(Vec2, Fac3)), v4_mul(Vec3, Fac4));
    or_v4 Inv2 = v4_add(v4_sub(v4_mul(Vec0, Fac1), v4_mul(Vec1, Fac3)), v4_mul(Vec3, Fac5));
    or_v4 Inv3 = v4_add(v4_sub(v4_mul(Vec0, Fac2), v4_mul(Vec1, Fac4)), v4_mul(Vec2, Fac5));
    or_v4 SignA = v4(+1, -1, +1, -1), SignB = v4(-1, +1, -1, +1);
    or_m4 Inverse;
    Inverse.c[0] = v4_mul(Inv0, SignA);
    Inverse.c[1] = v4_mul(Inv1, SignB);
    Inverse.c[2] = v4_mul(Inv2, SignA);
    Inverse.c[3] = v4_mul(Inv3, SignB);
    or_v4 Row0 = v4(Inverse.c[0].x, Inverse.c[1].x, Inverse.c[2].x, Inverse.c[3].x);
    or_v4 Dot0 = v4_mul(M.c[0], Row0);
    float Dot1 = (Dot0.x + Dot0.y) + (Dot0.z + Dot0.w);
    float OneOverDeterminant = 1.0f / Dot1;
    for (int i = 0; i < 4; ++i) Inverse.c[i] = v4s(Inverse.c[i], OneOverDeterminant);
    return Inverse;
#undef m
}

/* ================================ NIfTI-2 loader ======================================= */

/* BinaryLoader.cu:273-335: raw 540-byte header, then dim1*dim2*dim3 float32 at vox_offset.
 * Field offsets from nifti2.h:59-98 (packed). */
int or_nifti_load(const char* path, or_nifti* h, float** volume) {
    FILE* f = fopen(path, "rb");
    if (!f) return -1;
    unsigned char hdr[540];
    if (fread(hdr, 1, 540, f) != 540) { fclose(f); return -2; }
    memset(h, 0, sizeof(*h));
    memcpy(&h->sizeof_hdr, hdr + 0, 4);
    memcpy(&h->datatype, hdr + 12, 2);
    memcpy(&h->bitpix, hdr + 14, 2);
    memcpy(h->dim, hdr + 16, 64);
    memcpy(h->pixdim, hdr + 104, 64);
    memcpy(&h->vox_offset, hdr + 168, 8);
    memcpy(&h->scl_slope, hdr + 176, 8);
    memcpy(&h->scl_inter, hdr + 184, 8);
    memcpy(&h->cal_max, hdr + 192, 8);
    memcpy(&h->cal_min, hdr + 200, 8);
    if (h->sizeof_hdr != 540 && h->sizeof_hdr != 348) { fclose(f); return -3; }
    /* the reference multiplies the untrusted dims unchecked (BinaryLoader.cu:323); here a product
     * that overflows, a non-positive dim or an absurd size is refused (found by the ASan/UBSan
     * fuzz, tests/test_sanitize.py) */
    int64_t n = 0, n12 = 0;
    if (h->dim[1] <= 0 || h->dim[2] <= 0 || h->dim[3] <= 0 || __builtin_mul_overflow(h->dim[1], h->dim[2], &n12) ||
        __builtin_mul_overflow(n12, h->dim[3], &n) || n > ((int64_t)1 << 36) || h->vox_offset < 0) {
        fclose(f);
        return -4;
    }
    float* v = (float*)malloc((size_t)n * sizeof(float));
    if (!v) { fclose(f); return -5; }
    if (fseeko(f, (off_t)h->vox_offset, SEEK_SET) != 0 ||
        fread(v, sizeof(float), (size_t)n, f) != (size_t)n) {
        free(v); fclose(f); return -6;
    }
    fclose(f);
    *volume = v;
    return 0;
}

/* ================================ transfer function ==================================== */

/* TransferFunction.cu:19-23 with Material.cpp:25-43 colours. */
int or_default_tf(or_interval* t) {
    const or_interval d[4] = {
        {0.0f, 1.0f, {0.0f, 0.0f, 0.0f, 0.0f}},                                     /* empty  */
        {30.0f / 255.0f, 80.0f / 255.0f, {241.0f / 255.0f, 218.0f / 255.0f, 202.0f / 255.0f, 0.3f}}, /* bone */
        {140.0f / 255.0f, 160.0f / 255.0f, {124.0f / 255.0f, 9.0f / 255.0f, 42.0f / 255.0f, 0.3f}},  /* muscle */
        {105.0f / 255.0f, 120.0f / 255.0f, {223.0f / 255.0f, 155.0f / 255.0f, 141.0f / 255.0f, 0.7f}}, /* brain */
    };
    memcpy(t, d, sizeof(d));
    return 4;
}

/* TransferFunction.cu:46-55: default interval 0, last closed interval containing value wins. */
int or_tf_class(const or_interval* tf, int n, float value) {
    int r = 0;
    for (int i = 0; i < n; ++i)
        if (value >= tf[i].lo && value <= tf[i].hi) r = i;
    return r;
}

/* ================================ octree =============================================== */

static int is_leaf(const or_octree* o, uint64_t i) { return (uint32_t)o->nodes[i].depth == o->maximum_depth; }

/* Octree.cu:131-156 */
static void create_node(or_octree* o, uint64_t index, int depth, or_v3 lo, or_v3 up) {
    or_node* n = &o->nodes[index];
    n->depth = depth; n->maximum_value = 0.0f; n->minimum_value = 0.0f;
    n->lower[0] = lo.x; n->lower[1] = lo.y; n->lower[2] = lo.z;
    n->upper[0] = up.x; n->upper[1] = up.y; n->upper[2] = up.z;
    if (is_leaf(o, index)) return;
    or_v3 dist = v3_sub(up, lo);
    for (int x = 0; x < 2; ++x)
        for (int y = 0; y < 2; ++y)
            for (int z = 0; z < 2; ++z) {
                uint64_t child = 8 * index + (uint64_t)(x * 4 + y * 2 + z + 1);
                /* translate(x*d.x/2, y*d.y/2, z*d.y/2) * vec4(lower, 1)  (note: z uses d.y, :145) */
                or_m4 t = or_glm_translate(m4_identity(), v3(x * dist.x / 2, y * dist.y / 2, z * dist.y / 2));
                or_v4 cl4 = or_glm_mulv(t, v4(lo.x, lo.y, lo.z, 1.0f));
                or_v3 cl = v3(cl4.x, cl4.y, cl4.z);
                t = or_glm_translate(m4_identity(), v3(dist.x / 2, dist.y / 2, dist.y / 2));
                or_v4 cu4 = or_glm_mulv(t, v4(cl.x, cl.y, cl.z, 1.0f));
                create_node(o, child, depth + 1, cl, v3(cu4.x, cu4.y, cu4.z));
            }
}

/* Octree.cu:79-129 */
static void update_node(or_octree* o, uint64_t index) {
    or_node* node = &o->nodes[index];
    if (is_leaf(o, index)) {
        const float L = (float)o->longest_dimension;
        or_m4 sm = or_glm_scale(m4_identity(), v3(L, L, L));
        or_v4 r4 = or_glm_mulv(sm, v4(node->lower[0], node->lower[1], node->lower[2], 1.0f));
        or_v3 res = v3(r4.x, r4.y, r4.z);
        const float hL = (float)o->longest_dimension / 2.0f;
        const float h1 = (float)o->dim[0] / 2.0f, h2 = (float)o->dim[1] / 2.0f, h3 = (float)o->dim[2] / 2.0f;
        if (res.x >= hL - h1 && res.x < hL + h1 &&
            res.y >= hL - h2 && res.y < hL + h2 &&
            res.z >= hL - h3 && res.z < hL + h3) {
            /* (int)(res + d/2 - L/2) evaluated left to right in float */
            float fx = (float)(int)(res.x + h1 - hL);
            float fy = (float)(int)(res.y + h2 - hL);
            float fz = (float)(int)(res.z + h3 - hL);
            /* transformVector3Position, BinaryLoader.cu:234-238 (int64 arithmetic, int result) */
            int idx = (int)((int64_t)(int)fx * o->dim[1] * o->dim[2] + (int64_t)(int)fy * o->dim[2] + (int)fz);
            node->maximum_value = o->volume[idx];
            node->minimum_value = node->maximum_value;
        } else {
            node->maximum_value = 0.0f;
            node->minimum_value = 0.0f;
        }
        return;
    }
    for (int c = 1; c <= 8; ++c) update_node(o, 8 * index + c);
    for (int c = 1; c <= 8; ++c) {
        const or_node* ch = &o->nodes[8 * index + c];
        if (node->maximum_value < ch->maximum_value) node->maximum_value = ch->maximum_value;
        if (node->minimum_value > ch->minimum_value) node->minimum_value = ch->minimum_value;
    }
}

/* Octree.cu:30-53 */
int or_octree_build(or_octree* o, const float* volume, int64_t d1, int64_t d2, int64_t d3) {
    memset(o, 0, sizeof(*o));
    o->volume = volume;
    o->dim[0] = d1; o->dim[1] = d2; o->dim[2] = d3;
    uint32_t L = 0;
    for (int i = 0; i < 3; ++i)
        if (L < (uint32_t)o->dim[i]) L = (uint32_t)o->dim[i];
    o->longest_dimension = L;
    uint32_t D = 0;
    while (pow(2, D) < L) D++;
    o->maximum_depth = D;
    uint64_t n = 0;
    for (uint32_t p = 0; p < D + 1; ++p) n += (uint64_t)1 << (3 * p);
    o->number_of_nodes = n;
    o->nodes = (or_node*)malloc(n * sizeof(or_node));
    if (!o->nodes) return -1;
    create_node(o, 0, 0, v3(0, 0, 0), v3(1, 1, 1));
    update_node(o, 0);
    return 0;
}

void or_octree_free(or_octree* o) { free(o->nodes); o->nodes = NULL; }

/* Same L and D as or_octree_build, no node pool: or_octree_intensity then evaluates the closed form
 * of the search, which tests/test_oracle_pin.py checks against the literal
 * tree on every leaf.  For volumes whose node pool cannot exist (512^3: 5.5 GB, 2048^3: 353 GB).
 * Voxel indices are int64: the reference's int index (BinaryLoader.cu:234-238) overflows beyond
 * 2^31 voxels, where its behaviour is undefined. */
int or_octree_init_implicit(or_octree* o, const float* volume, int64_t d1, int64_t d2, int64_t d3) {
    memset(o, 0, sizeof(*o));
    o->volume = volume;
    o->dim[0] = d1; o->dim[1] = d2; o->dim[2] = d3;
    uint32_t L = 0;
    for (int i = 0; i < 3; ++i)
        if (L < (uint32_t)o->dim[i]) L = (uint32_t)o->dim[i];
    o->longest_dimension = L;
    uint32_t D = 0;
    while (pow(2, D) < L) D++;
    o->maximum_depth = D;
    o->number_of_nodes = 0;
    return 0;
}

static int leaf_voxel(const or_octree* o, const float q[3], int v[3]);

/* Octree.cu:257-269 */
static inline int node_inside(const or_node* n, float px, float py, float pz) {
    return px >= n->lower[0] && py >= n->lower[1] && pz >= n->lower[2] &&
           px < n->upper[0] && py < n->upper[1] && pz < n->upper[2];
}

/* Octree.cu:162-183 */
static float search(const or_octree* o, uint64_t index, float px, float py, float pz) {
    float res = 0.0f;
    const or_node* n = &o->nodes[index];
    if (node_inside(n, px, py, pz)) {
        if (n->maximum_value == n->minimum_value) {
            res = n->maximum_value;
        } else {
            for (int c = 1; c <= 8; ++c) {
                float aux = search(o, index * 8 + c, px, py, pz);
                if (aux > res) res = aux;
            }
        }
    }
    return res;
}

float or_octree_intensity(const or_octree* o, float qx, float qy, float qz) {
    if (o->nodes) return search(o, 0, qx, qy, qz);
    const float q[3] = {qx, qy, qz};
    int v[3];
    if (!leaf_voxel(o, q, v)) return 0.0f;
    const float x = o->volume[(int64_t)v[0] * o->dim[1] * o->dim[2] + (int64_t)v[1] * o->dim[2] + v[2]];
    return x > 0.0f ? x : 0.0f;
}

void or_octree_leaf_values(const or_octree* o, float* out, int threads) {
    const int64_t n = (int64_t)1 << o->maximum_depth;
    const float inv = 1.0f / (float)n;
#ifdef _OPENMP
    if (threads <= 0) threads = omp_get_max_threads();
#pragma omp parallel for schedule(dynamic, 1) num_threads(threads)
#endif
    for (int64_t ix = 0; ix < n; ++ix)
        for (int64_t iy = 0; iy < n; ++iy)
            for (int64_t iz = 0; iz < n; ++iz)
                out[(ix * n + iy) * n + iz] = or_octree_intensity(o, (float)ix * inv, (float)iy * inv, (float)iz * inv);
    (void)threads;
}

/* ================================ camera / params ====================================== */

void or_camera_derive(const float pos[3], const float up_in[3], float rsw, float rsh, or_camera* c) {
    /* myApp.cu:1105-1112 with rotationMat = translationMat = identity */
    or_m4 I = m4_identity();
    or_m4 rt = or_glm_mul(I, I);
    or_v4 p4 = or_glm_mulv(rt, v4(pos[0], pos[1], pos[2], 1.0f));
    or_v3 p = v3(p4.x, p4.y, p4.z);
    or_v3 up = v3(up_in[0], up_in[1], up_in[2]);
    or_v3 front = or_glm_normalize(v3_sub(v3(0, 0, 0), p));
    or_v3 right = or_glm_normalize(or_glm_cross(up, front));
    up = or_glm_cross(front, right);
    or_v3 tlc = v3_add(v3_add(p, sv3(rsw / 2, v3_neg(right))), v3s(up, rsh / 2));
    c->pos[0] = p.x; c->pos[1] = p.y; c->pos[2] = p.z;
    c->front[0] = front.x; c->front[1] = front.y; c->front[2] = front.z;
    c->right[0] = right.x; c->right[1] = right.y; c->right[2] = right.z;
    c->up[0] = up.x; c->up[1] = up.y; c->up[2] = up.z;
    c->top_left[0] = tlc.x; c->top_left[1] = tlc.y; c->top_left[2] = tlc.z;
}

void or_camera_derive_conic(const float pos[3], const float up[3], float rsw, float rsh, float vpd, or_camera* c) {
    or_camera_derive(pos, up, rsw, rsh, c);
    or_v3 p = cam_v(c->pos), front = cam_v(c->front), right = cam_v(c->right), u = cam_v(c->up);
    or_v3 tlc = v3_add(v3_add(v3_add(p, sv3(vpd, front)), sv3(rsw / 2, v3_neg(right))), v3s(u, rsh / 2));
    c->top_left[0] = tlc.x; c->top_left[1] = tlc.y; c->top_left[2] = tlc.z;
}

void or_point_cloud(const float* vol, int64_t d1, int64_t d2, int64_t d3, double cal_max, const or_interval* tf,
                    int n_tf, float* out) {
    int L = 0;   /* myApp.cu:1283-1287 */
    const int64_t d[3] = {d1, d2, d3};
    for (int i = 0; i < 3; ++i)
        if (d[i] > L) L = (int)d[i];
    const float vd[3] = {(float)d1, (float)d2, (float)d3};   /* volume_dimensions (float[]) */
    for (int64_t x = 0; x < d1; ++x)
        for (int64_t y = 0; y < d2; ++y)
            for (int64_t z = 0; z < d3; ++z) {
                const int64_t vi = (x * d2 + y) * d3 + z;
                float* o = out + vi * 7;
                o[0] = (((float)x + L / 2.0f) - (vd[0] / 2.0f)) / L;
                o[1] = (((float)y + L / 2.0f) - (vd[1] / 2.0f)) / L;
                o[2] = (((float)z + L / 2.0f) - (vd[2] / 2.0f)) / L;
                const int k = or_tf_class(tf, n_tf, (float)(vol[vi] / cal_max));
                memcpy(o + 3, tf[k].rgba, 16);
            }
}

void or_params_default(int W, int H, int S, or_params* p) {
    /* utils.h:53-74 */
    float view_angle = (float)(M_PI / 4);
    p->width = W; p->height = H; p->samples_per_ray = S;
    p->viewplane_distance = 2.0f;
    p->real_screen_width = 2 * tanf(view_angle);
    p->real_screen_height = p->real_screen_width * (float)(unsigned)H / (float)(unsigned)W;
    p->front_clip_plane = 0.0f;
    p->sample_distance = (p->viewplane_distance - p->front_clip_plane) / (float)(unsigned)S;
    p->background[0] = 0.2f; p->background[1] = 0.2f; p->background[2] = 0.2f; p->background[3] = 1.0f;
    p->conic = 0;
}

void or_camera_default(int W, int H, or_camera* c) {
    or_params p;
    or_params_default(W, H, 1, &p);
    /* utils.h:41-46 initialisers */
    or_v3 pos = v3(0.0f, 0.0f, 1.0f);
    or_v3 front = or_glm_normalize(v3_sub(v3(0, 0, 0), pos));
    or_v3 up0 = v3(0.0f, 1.0f, 0.0f);
    or_v3 right = or_glm_normalize(or_glm_cross(front, up0));
    or_v3 up = or_glm_normalize(or_glm_cross(right, front));
    float P[3] = {pos.x, pos.y, pos.z}, U[3] = {up.x, up.y, up.z};
    or_camera_derive(P, U, p.real_screen_width, p.real_screen_height, c);
}

void or_camera_oblique(int W, int H, or_camera* c) {
    /* utils.h:77-81, applied raw by resetCameraAttributes (myApp.cu:1911-1917) AFTER that
     * frame's derivation, so the re-rendered frame sees these exact vectors. */
    (void)W; (void)H;
    const float pos[3] = {0.456607f, 0.693644f, (float)-0.55711};
    const float fr[3] = {-0.456606f, -0.693643f, 0.557109f};
    const float ri[3] = {-0.19427f, -0.533349f, -0.823285f};
    const float up[3] = {0.868199f, -0.484147f, 0.108777f};
    const float tl[3] = {1.51908f, 0.742847f, 0.374952f};
    memcpy(c->pos, pos, 12); memcpy(c->front, fr, 12); memcpy(c->right, ri, 12);
    memcpy(c->up, up, 12); memcpy(c->top_left, tl, 12);
}

/* ================================ VRC =================================================== */


/* kernel.cu:53-59 (orthographic branch; device_primary_rays[...] == cameraFront, :36) and the
 * modelAux = translate(mat4(1), vec3(0.5)) product (kernel.cu:1050, :62). */
void or_vrc_sample_point(const or_params* p, const or_camera* c, int x, int y, int s, float q[3]) {
    or_v3 tlc = cam_v(c->top_left), right = cam_v(c->right), up = cam_v(c->up), dir = cam_v(c->front);
    float a = (float)x * p->real_screen_width / (float)(unsigned)p->width;
    float b = (float)y * p->real_screen_height / (float)(unsigned)p->height;
    float t = (float)s * p->sample_distance + p->front_clip_plane;
    or_v3 pos;
    if (p->conic) {
        /* kernel.cu:30-34 (ray direction) and :53-54 (sample position) */
        or_v3 eye = cam_v(c->pos);
        or_v3 d = or_glm_normalize(v3_sub(v3_add(v3_add(tlc, sv3(a, right)), sv3(b, v3_neg(up))), eye));
        pos = v3_add(eye, sv3(t, d));
    } else {
        pos = v3_add(v3_add(v3_add(tlc, sv3(a, right)), sv3(b, v3_neg(up))), sv3(t, dir));
    }
    or_m4 model = or_glm_translate(m4_identity(), v3(0.5f, 0.5f, 0.5f));
    or_v4 r = or_glm_mulv(model, v4(pos.x, pos.y, pos.z, 1.0f));
    q[0] = r.x; q[1] = r.y; q[2] = r.z;
}

static inline void vrc_sample_rgba(const or_octree* o, int max_intensity, const or_interval* tf, int n_tf,
                                   const or_params* p, const or_camera* c, int x, int y, int s, float rgba[4]) {
    float q[3];
    or_vrc_sample_point(p, c, x, y, s, q);
    /* kernel.cu:64: octree intensity / (int)cal_max (float / int) */
    float n = or_octree_intensity(o, q[0], q[1], q[2]) / (float)max_intensity;
    const or_interval* m = &tf[or_tf_class(tf, n_tf, n)];
    memcpy(rgba, m->rgba, 16);
}

/* kernel.cu:194-225: back to front over s = S-1..0, alpha forced to 1. */
static inline void blend(float f[4], const float c[4]) {
    f[0] = f[0] * (1 - c[3]) + c[0] * c[3];
    f[1] = f[1] * (1 - c[3]) + c[1] * c[3];
    f[2] = f[2] * (1 - c[3]) + c[2] * c[3];
    f[3] = 1.0f;
}

void or_vrc_ray_samples(const or_octree* o, double cal_max, const or_interval* tf, int n_tf,
                        const or_params* p, const or_camera* c, int x, int y, float* out) {
    int mi = (int)cal_max;   /* kernel.cu:1151: double cal_max passed as int max_intensity */
    for (int s = 0; s < p->samples_per_ray; ++s)
        vrc_sample_rgba(o, mi, tf, n_tf, p, c, x, y, s, out + 4 * (size_t)s);
}

void or_render_vrc_columns(const or_octree* o, double cal_max, const or_interval* tf, int n_tf,
                           const or_params* p, const or_camera* c, const int* xs, int nx, float* out, int threads) {
    const int H = p->height, S = p->samples_per_ray;
    const int mi = (int)cal_max;
#ifdef _OPENMP
    if (threads <= 0) threads = omp_get_max_threads();
#pragma omp parallel for schedule(dynamic, 1) num_threads(threads)
#endif
    for (int i = 0; i < nx; ++i) {
        const int x = xs ? xs[i] : i;
        for (int y = 0; y < H; ++y) {
            float f[4] = {p->background[0], p->background[1], p->background[2], p->background[3]};
            for (int s = S - 1; s >= 0; --s) {
                float rgba[4];
                vrc_sample_rgba(o, mi, tf, n_tf, p, c, x, y, s, rgba);
                blend(f, rgba);
            }
            memcpy(out + 4 * ((size_t)i * H + y), f, 16);
        }
    }
    (void)threads;
}

void or_render_vrc(const or_octree* o, double cal_max, const or_interval* tf, int n_tf,
                   const or_params* p, const or_camera* c, float* out, int threads) {
    or_render_vrc_columns(o, cal_max, tf, n_tf, p, c, NULL, p->width, out, threads);
}

/* Voxel of the leaf containing q (Octree.cu:85-100), or 0 if q is outside the cube / dataset. */
static int leaf_voxel(const or_octree* o, const float q[3], int v[3]) {
    for (int a = 0; a < 3; ++a)
        if (!(q[a] >= 0.0f && q[a] < 1.0f)) return 0;
    const float scale = (float)((uint64_t)1 << o->maximum_depth);
    const float L = (float)o->longest_dimension, hL = L / 2.0f;
    for (int a = 0; a < 3; ++a) {
        float lc = floorf(q[a] * scale) / scale;
        float res = L * lc;
        float h = (float)o->dim[a] / 2.0f;
        if (!(res >= hL - h && res < hL + h)) return 0;
        v[a] = (int)(res + h - hL);
    }
    return 1;
}

/* The shading stage (see vr_kernels.hip shade_sample; same operations, same order). */
static void or_shade(const or_octree* o, const int v[3], const float Lh[3], const float sh[4], float rgb[3]) {
    const int64_t d1 = o->dim[0], d2 = o->dim[1], d3 = o->dim[2];
    const int64_t sx = d2 * d3, sy = d3;
    const int64_t c = (int64_t)v[0] * sx + (int64_t)v[1] * sy + v[2];
    const float* vol = o->volume;
    const float gx = (vol[c + (v[0] + 1 < d1 ? sx : 0)] - vol[c - (v[0] > 0 ? sx : 0)]) * 0.5f;
    const float gy = (vol[c + (v[1] + 1 < d2 ? sy : 0)] - vol[c - (v[1] > 0 ? sy : 0)]) * 0.5f;
    const float gz = (vol[c + (v[2] + 1 < d3 ? 1 : 0)] - vol[c - (v[2] > 0 ? 1 : 0)]) * 0.5f;
    const float len2 = (gx * gx + gy * gy) + gz * gz;
    float d = 1.0f, spec = 0.0f;
    if (len2 > 0.0f) {
        const float inv = 1.0f / sqrtf(len2);
        const float ndl = ((-gx * inv) * Lh[0] + (-gy * inv) * Lh[1]) + (-gz * inv) * Lh[2];
        d = ndl > 0.0f ? ndl : 0.0f;
        /* d^shininess as exp2(shininess * log2 d), d > 0 (the kernel's hardware v_exp/v_log agree to
         * a few ulp); d = 0 -> 0 (shininess 0 -> 1) */
        spec = d > 0.0f ? sh[2] * exp2f(sh[3] * log2f(d)) : (sh[3] == 0.0f ? sh[2] : 0.0f);
    }
    const float k = sh[0] + sh[1] * d;
    for (int i = 0; i < 3; ++i) rgb[i] = rgb[i] * k + spec;
}

void or_render_vrc_shaded(const or_octree* o, double cal_max, const or_interval* tf, int n_tf,
                          const or_params* p, const or_camera* c, const float sh[4], float* out, int threads) {
    const int W = p->width, H = p->height, S = p->samples_per_ray;
    const int mi = (int)cal_max;
    const float Lh[3] = {-c->front[0], -c->front[1], -c->front[2]};
#ifdef _OPENMP
    if (threads <= 0) threads = omp_get_max_threads();
#pragma omp parallel for schedule(dynamic, 1) num_threads(threads)
#endif
    for (int x = 0; x < W; ++x) {
        for (int y = 0; y < H; ++y) {
            float f[4] = {p->background[0], p->background[1], p->background[2], p->background[3]};
            for (int s = S - 1; s >= 0; --s) {
                float q[3], rgba[4];
                or_vrc_sample_point(p, c, x, y, s, q);
                float n = or_octree_intensity(o, q[0], q[1], q[2]) / (float)mi;
                memcpy(rgba, tf[or_tf_class(tf, n_tf, n)].rgba, 16);
                int v[3];
                if (rgba[3] != 0.0f && leaf_voxel(o, q, v)) or_shade(o, v, Lh, sh, rgba);
                blend(f, rgba);
            }
            memcpy(out + 4 * ((size_t)x * H + y), f, 16);
        }
    }
    (void)threads;
}

/* Leaf-in-dataset test of Octree.cu:91-94 for query point q (N_in of SURVEY 8(d)). */
static int in_dataset(const or_octree* o, const float q[3]) {
    for (int a = 0; a < 3; ++a)
        if (!(q[a] >= 0.0f && q[a] < 1.0f)) return 0;
    const float scale = (float)((uint64_t)1 << o->maximum_depth);
    const float L = (float)o->longest_dimension, hL = L / 2.0f;
    for (int a = 0; a < 3; ++a) {
        float lc = floorf(q[a] * scale) / scale;
        float res = L * lc;
        float h = (float)o->dim[a] / 2.0f;
        if (!(res >= hL - h && res < hL + h)) return 0;
    }
    return 1;
}

uint64_t or_count_in_samples(const or_octree* o, const or_params* p, const or_camera* c, int threads) {
    const int W = p->width, H = p->height, S = p->samples_per_ray;
    uint64_t total = 0;
#ifdef _OPENMP
    if (threads <= 0) threads = omp_get_max_threads();
#pragma omp parallel for schedule(dynamic, 1) num_threads(threads) reduction(+ : total)
#endif
    for (int x = 0; x < W; ++x)
        for (int y = 0; y < H; ++y)
            for (int s = 0; s < S; ++s) {
                float q[3];
                or_vrc_sample_point(p, c, x, y, s, q);
                total += (uint64_t)in_dataset(o, q);
            }
    (void)threads;
    return total;
}

/* ================================ TEST ================================================== */

void or_test_matrices(int64_t d1, int64_t d2, int64_t d3, const or_params* p, const or_camera* c,
                      or_m4* model_cam, or_m4* inverse_view, or_m4* to_volume) {
    /* kernel.cu:1177-1190 */
    or_m4 mc = or_glm_translate(m4_identity(), v3(-p->real_screen_width / 2.0f, -p->real_screen_height / 2.0f, 0.0f));
    mc = or_glm_scale(mc, v3(p->real_screen_width / (float)(unsigned)p->width,
                             p->real_screen_height / (float)(unsigned)p->height,
                             -p->viewplane_distance / (float)(unsigned)p->samples_per_ray));
    /* kernel.cu:1194-1195 */
    or_m4 view = or_glm_lookat(cam_v(c->pos), v3(0, 0, 0), cam_v(c->up));
    view = or_glm_inverse(view);
    /* kernel.cu:1200-1216; longest_dimension = max(dim) (BinaryLoader.cu:33-36) */
    int64_t Ld = d1 > d2 ? d1 : d2;
    if (d3 > Ld) Ld = d3;
    int L = (int)Ld;
    or_m4 tv = m4_identity();
    or_m4 t1 = or_glm_translate(m4_identity(), v3(0.5f, 0.5f, 0.5f));
    or_m4 sc = or_glm_scale(m4_identity(), v3((float)L, (float)L, (float)L));
    or_m4 t2 = or_glm_translate(m4_identity(), v3((float)d1 / 2.0f - (float)L / 2.0f,
                                                  (float)d2 / 2.0f - (float)L / 2.0f,
                                                  (float)d3 / 2.0f - (float)L / 2.0f));
    tv = or_glm_mul(t1, tv);
    tv = or_glm_mul(sc, tv);
    tv = or_glm_mul(t2, tv);
    *model_cam = mc; *inverse_view = view; *to_volume = tv;
}

static inline or_v4 lerp4(or_v4 a, or_v4 b, float w) {
    /* a * (1 - w) + b * w  (kernel.cu:162-175) */
    return v4_add(v4s(a, 1.0f - w), v4s(b, w));
}

void or_render_test(const float* vol, int64_t d1, int64_t d2, int64_t d3, double cal_max,
                    const or_interval* tf, int n_tf, const or_params* p, const or_camera* c,
                    float* out, int threads) {
    or_render_test_columns(vol, d1, d2, d3, cal_max, tf, n_tf, p, c, NULL, p->width, out, threads);
}

/* Columns xs[0..nx) of the TEST frame (xs == NULL: columns 0..nx), out[(i*H + y)*4 + c]: the
 * frame's [x*H + y] layout restricted to the listed columns (C3-size parity samples). */
void or_render_test_columns(const float* vol, int64_t d1, int64_t d2, int64_t d3, double cal_max,
                            const or_interval* tf, int n_tf, const or_params* p, const or_camera* c,
                            const int* xs, int nx, float* out, int threads) {
    const int H = p->height, S = p->samples_per_ray;
    or_m4 mc, iv, tv;
    or_test_matrices(d1, d2, d3, p, c, &mc, &iv, &tv);
    const int totaldim = (int)(d1 * d2 * d3);   /* setTotalDim, BinaryLoader.cu:409-415 */
    const float* col0 = tf[or_tf_class(tf, n_tf, (float)(0.0f / cal_max))].rgba;
#ifdef _OPENMP
    if (threads <= 0) threads = omp_get_max_threads();
#pragma omp parallel for schedule(dynamic, 1) num_threads(threads)
#endif
    for (int i = 0; i < nx; ++i) {
        const int x = xs ? xs[i] : i;
        for (int y = 0; y < H; ++y) {
            float f[4] = {p->background[0], p->background[1], p->background[2], p->background[3]};
            for (int s = S - 1; s >= 0; --s) {
                /* kernel.cu:100-115: three successive mat*vec, each truncated to vec3 */
                or_v4 q = or_glm_mulv(mc, v4((float)x, (float)y, (float)s, 1.0f));
                q = or_glm_mulv(iv, v4(q.x, q.y, q.z, 1.0f));
                q = or_glm_mulv(tv, v4(q.x, q.y, q.z, 1.0f));
                or_v4 cf = v4(col0[0], col0[1], col0[2], col0[3]);
                /* NiftiFile::isInside, BinaryLoader.cu:240-245 */
                if (q.x >= 0.0f && q.x < (float)d1 && q.y >= 0.0f && q.y < (float)d2 && q.z >= 0.0f && q.z < (float)d3) {
                    or_v4 cc[8];
                    for (int k = 0; k < 8; ++k) {
                        /* corner order kernel.cu:124-158: (0,0,0),(0,0,1),(0,1,0),(0,1,1),(1,0,0),... */
                        float ox = (float)((k >> 2) & 1), oy = (float)((k >> 1) & 1), oz = (float)(k & 1);
                        float cx = q.x + ox, cy = q.y + oy, cz = q.z + oz;
                        int idx = (int)((int64_t)(int)cx * d2 * d3 + (int64_t)(int)cy * d3 + (int)cz);
                        float v = (idx < totaldim) ? vol[idx] : 0.0f;
                        const float* m = tf[or_tf_class(tf, n_tf, (float)(v / cal_max))].rgba;
                        cc[k] = v4(m[0], m[1], m[2], m[3]);
                    }
                    float dx = q.x - (float)(int)q.x, dy = q.y - (float)(int)q.y, dz = q.z - (float)(int)q.z;
                    or_v4 y1 = lerp4(cc[0], cc[2], dy);
                    or_v4 y2 = lerp4(cc[1], cc[3], dy);
                    or_v4 y3 = lerp4(cc[4], cc[6], dy);
                    or_v4 y4 = lerp4(cc[5], cc[7], dy);
                    or_v4 z1 = lerp4(y1, y3, dx);
                    or_v4 z2 = lerp4(y2, y4, dx);
                    cf = lerp4(z1, z2, dz);
                }
                float rgba[4] = {cf.x, cf.y, cf.z, cf.w};
                blend(f, rgba);
            }
            memcpy(out + 4 * ((size_t)i * H + y), f, 16);
        }
    }
    (void)threads;
}

/* ================================ CPU ray-cast path (baseline) ========================= */

void or_render_cpu_path(const or_octree* o, double cal_max, const or_interval* tf, int n_tf,
                        const or_params* p, const or_camera* c, int x0, int x1, float* out, int threads) {
    or_render_cpu_path_columns(o, cal_max, tf, n_tf, p, c, NULL, x0, x1 - x0, out, threads);
}

void or_render_cpu_path_columns(const or_octree* o, double cal_max, const or_interval* tf, int n_tf,
                                const or_params* p, const or_camera* c, const int* xs, int x0, int nx, float* out,
                                int threads) {
    const int H = p->height, S = p->samples_per_ray;
    /* myApp.cu:1406-1409 */
    const float deg2rad = (float)0.01745329251994329576923690768489;
    or_m4 model = or_glm_translate(m4_identity(), v3(0.5f, 0.5f, 0.5f));
    model = or_glm_rotate(model, 90.0f * deg2rad, v3(0.0f, 1.0f, 0.0f));
    model = or_glm_rotate(model, 90.0f * deg2rad, v3(-1.0f, 0.0f, 0.0f));
    or_v3 tlc = cam_v(c->top_left), right = cam_v(c->right), up = cam_v(c->up), dir = cam_v(c->front);
#ifdef _OPENMP
    if (threads <= 0) threads = omp_get_max_threads();
#pragma omp parallel for schedule(dynamic, 1) num_threads(threads)
#endif
    for (int k = 0; k < nx; ++k) {
        const int x = xs ? xs[k] : x0 + k;
        for (int y = 0; y < H; ++y) {
            float f[4] = {p->background[0], p->background[1], p->background[2], p->background[3]};
            for (int i = S; i > 0; --i) {   /* myApp.cu:1445 */
                float a = (float)x * p->real_screen_width / (float)(unsigned)p->width;
                float b = (float)y * p->real_screen_height / (float)(unsigned)p->height;
                float t = (float)i * p->sample_distance;
                or_v3 pos = v3_add(v3_add(v3_add(tlc, sv3(a, right)), sv3(b, v3_neg(up))), sv3(t, dir));
                or_v4 q = or_glm_mulv(model, v4(pos.x, pos.y, pos.z, 1.0f));
                float I = or_octree_intensity(o, q.x, q.y, q.z);
                float n = (float)(I / cal_max);   /* myApp.cu:1463: double cal_max */
                blend(f, tf[or_tf_class(tf, n_tf, n)].rgba);
            }
            memcpy(out + 4 * ((size_t)k * H + y), f, 16);
        }
    }
    (void)threads;
}

/* ============================ synthetic C5 volume =========================== */

static uint64_t splitmix64(uint64_t x) {
    uint64_t z = x + 0x9E3779B97F4A7C15ull;
    z = (z ^ (z >> 30)) * 0xBF58476D1CE4E5B9ull;
    z = (z ^ (z >> 27)) * 0x94D049BB133111EBull;
    return z ^ (z >> 31);
}

float or_synthetic_voxel(int64_t n, uint64_t seed, int64_t x, int64_t y, int64_t z) {
    const double c = (double)(n - 1) / 2.0;
    const double dx = (double)x - c, dy = (double)y - c, dz = (double)z - c;
    const double r = sqrt(dx * dx + dy * dy + dz * dz) / ((double)n / 2.0);
    if (!(r < 0.95)) return 0.0f;
    const double w = round(127.5 + 127.5 * sin(16.0 * M_PI * r));
    const int64_t idx = (x * n + y) * n + z;
    const int64_t noise = (int64_t)(splitmix64(seed ^ (uint64_t)idx) % 17u) - 8;
    int64_t v = (int64_t)w + noise;
    v = v < 0 ? 0 : (v > 255 ? 255 : v);
    return (float)v;
}

void or_synthetic_slab(int64_t n, uint64_t seed, int64_t x0, int64_t nx, float* out, int threads) {
#ifdef _OPENMP
    if (threads <= 0) threads = omp_get_max_threads();
#pragma omp parallel for schedule(static) num_threads(threads)
#endif
    for (int64_t i = 0; i < nx * n; ++i) {
        const int64_t x = x0 + i / n, y = i % n;
        for (int64_t z = 0; z < n; ++z) out[i * n + z] = or_synthetic_voxel(n, seed, x, y, z);
    }
    (void)threads;
}

/* ================================ FP-contraction sensitivity ============================= */
/* The restatement (and libvr) evaluate the reference's arithmetic as written, every product and
 * sum rounded.  nvcc's default (-fmad=true) may fuse a*b + c in the reference's own device build;
 * which pairs it fuses is the compiler's choice, so the model below fuses every a*b + c of the
 * position expressions (kernel.cu:55-59 VRC; the three glm mat4*vec4 of kernel.cu:100-115 TEST)
 * and counts the samples whose octree leaf (VRC) or corner voxels / inside test (TEST) change --
 * the samples the two models can disagree on.  Test infrastructure only. */
uint64_t or_vrc_contraction_flips(const or_octree* o, const or_params* p, const or_camera* c, uint64_t* n_in) {
    const int W = p->width, H = p->height, S = p->samples_per_ray;
    const float scale = (float)((uint64_t)1 << o->maximum_depth);
    uint64_t flips = 0, nin = 0;
    for (int x = 0; x < W; ++x)
        for (int y = 0; y < H; ++y)
            for (int s = 0; s < S; ++s) {
                float q[3];
                or_vrc_sample_point(p, c, x, y, s, q);
                const float a = (float)x * p->real_screen_width / (float)(unsigned)W;
                const float b = (float)y * p->real_screen_height / (float)(unsigned)H;
                const float t = fmaf((float)s, p->sample_distance, p->front_clip_plane);
                float qf[3];
                for (int k = 0; k < 3; ++k) {
                    const float pos = fmaf(t, c->front[k], fmaf(b, -c->up[k], fmaf(a, c->right[k], c->top_left[k])));
                    qf[k] = pos + 0.5f;
                }
                const int in0 = in_dataset(o, q), in1 = in_dataset(o, qf);
                if (!in0 && !in1) continue;
                ++nin;
                int diff = in0 != in1;
                for (int k = 0; k < 3 && !diff; ++k) diff = floorf(q[k] * scale) != floorf(qf[k] * scale);
                flips += (uint64_t)diff;
            }
    if (n_in) *n_in = nin;
    return flips;
}

static or_v4 mulv_fused(or_m4 m, or_v4 v) {
    /* glm (m0 x + m1 y) + (m2 z + m3 w), each inner pair fused */
    const float* a = &m.c[0].x;   /* column-major, 16 floats */
    float r[4];
    for (int k = 0; k < 4; ++k)
        r[k] = fmaf(a[4 + k], v.y, a[k] * v.x) + fmaf(a[12 + k], v.w, a[8 + k] * v.z);
    return v4(r[0], r[1], r[2], r[3]);
}

uint64_t or_test_contraction_flips(int64_t d1, int64_t d2, int64_t d3, const or_params* p, const or_camera* c,
                                   uint64_t* n_in) {
    const int W = p->width, H = p->height, S = p->samples_per_ray;
    or_m4 mc, iv, tv;
    or_test_matrices(d1, d2, d3, p, c, &mc, &iv, &tv);
    uint64_t flips = 0, nin = 0;
    for (int x = 0; x < W; ++x)
        for (int y = 0; y < H; ++y)
            for (int s = 0; s < S; ++s) {
                or_v4 q = or_glm_mulv(mc, v4((float)x, (float)y, (float)s, 1.0f));
                q = or_glm_mulv(iv, v4(q.x, q.y, q.z, 1.0f));
                q = or_glm_mulv(tv, v4(q.x, q.y, q.z, 1.0f));
                or_v4 f = mulv_fused(mc, v4((float)x, (float)y, (float)s, 1.0f));
                f = mulv_fused(iv, v4(f.x, f.y, f.z, 1.0f));
                f = mulv_fused(tv, v4(f.x, f.y, f.z, 1.0f));
                const float a[3] = {q.x, q.y, q.z}, b[3] = {f.x, f.y, f.z}, dim[3] = {(float)d1, (float)d2, (float)d3};
                int ina = 1, inb = 1;
                for (int k = 0; k < 3; ++k) {
                    ina &= a[k] >= 0.0f && a[k] < dim[k];
                    inb &= b[k] >= 0.0f && b[k] < dim[k];
                }
                if (!ina && !inb) continue;
                ++nin;
                int diff = ina != inb;
                for (int k = 0; k < 3 && !diff; ++k)
                    diff = (int)a[k] != (int)b[k] || (int)(a[k] + 1.0f) != (int)(b[k] + 1.0f);
                flips += (uint64_t)diff;
            }
    if (n_in) *n_in = nin;
    return flips;
}
