/*
 * physics_oracle.c -- TEST INFRASTRUCTURE ONLY (never linked into the product).
 *
 * CPU restatement, in plain C, of one `gym.simulate()` call of the build's
 * articulation + plane-contact solver.  It is the checker the HIP kernels in
 * isaacgymenv_amd/csrc/ are compared against; only tests/, __graft_entry__.smoke()
 * and bench.py's cpu_baseline leg may load it.
 *
 * PARITY STATUS vs the reference: UNPINNED.  The reference's physics is the
 * closed Isaac Gym / PhysX binary called at vec_task.py:382 and
 * anymal_terrain.py:448; it is neither in
 * /root/reference nor installable here.  This file restates the *solver
 * specification written in DESIGN.md section 3*, which follows the config
 * semantics the reference hands PhysX:
 *   dt / substeps                     AnymalTerrain.yaml:129-131, vec_task.py:532-535
 *   num_position/velocity_iterations  AnymalTerrain.yaml:138-139
 *   contact_offset / rest_offset      AnymalTerrain.yaml:140-141
 *   max_depenetration_velocity        AnymalTerrain.yaml:143
 *   contact_collection (last substep) AnymalTerrain.yaml:146
 *   ground friction / restitution     anymal_terrain.py:188-194
 *   per-shape friction buckets        anymal_terrain.py:236-281
 *   effort limit / velocity limit     anymal_minimal.urdf <limit effort velocity>
 *   joint limits                      nv_ant.xml <joint range limited="true"> (Ant.yaml)
 *   force sensors (leaf bodies)       ant.py:174-178, 233-235
 *
 * The formulation here is deliberately different from the kernels: generic
 * runtime topology, dense CRBA mass matrix, dense Cholesky, joint-space
 * sequential impulses with W = M^-1 J^T.  The kernels use compile-time
 * topology, the tree-sparse L^T D L factorisation and a w-space PGS.  Both
 * produce the same iterates in exact arithmetic.
 *
 * REAL is double by default (the oracle); -DREAL=float builds the fp32
 * CPU baseline (bench.py cpu_baseline, kind "port").
 */
#include <math.h>
#include <stdint.h>
#include <stdio.h>
#include <stdlib.h>
#include <string.h>
#ifdef _OPENMP
#include <omp.h>
#endif

#ifndef REAL
#define REAL double
#endif
typedef REAL real;
/* GJK's convergence bound on vv - v.w relative to vv: 1e-10 in fp64; the fp32 build uses the float kernels' 1e-6
 * (gs_pairs.h gjk_cores: below ~1e-7 vv a float test reads rounding, and a search that cannot stop runs into a
 * degenerate 4-point simplex that reads as overlapping cores -- not the rounding of the spec, a failure of it) */
#define GJK_TOL (sizeof(real) == sizeof(double) ? 1e-10 : 1e-6)

#define MAXB 32
#define MAXV 40
#define MAXC 192
#define MAXPOOL 16
#define MIN_RESPONSE 1e-3 /* a self-contact row whose J M^-1 J^T falls below this (an effective mass above 1000 kg:
                             an overlap no dof can separate) takes no impulse (GS_MIN_RESPONSE); ground rows
                             always respond */

typedef struct {
    int32_t nb, nd, nc, ns, fixed_base;
    const int32_t *parent;      /* [nb] */
    const int32_t *jkind;       /* [nb] 1 revolute 2 prismatic (root: 3 free / 0 fixed) */
    const int32_t *bdof;        /* [nb] dof index of the body's joint, -1 for the root */
    const double *jorigin;      /* [nb][12] R row-major (9) + t (3) */
    const double *jaxis;        /* [nb][3] */
    const double *mass;         /* [nb] */
    const double *com;          /* [nb][3] */
    const double *inertia;      /* [nb][9] about COM */
    const int32_t *cbody;       /* [nc] */
    const double *cpoint;       /* [nc][3] */
    const double *cradius;      /* [nc] */
    const int32_t *cshape;      /* [nc] */
    const double *effort;       /* [nd] <= 0 : unlimited */
    const double *vmax;         /* [nd] <= 0 : unlimited */
    const double *armature;     /* [nd] */
    const double *lower;        /* [nd] joint limits where has_limits */
    const double *upper;        /* [nd] */
    const int32_t *has_limits;  /* [nd] */
    int32_t nsens;              /* force sensors */
    const int32_t *sens_body;   /* [nsens] leaf bodies */
    int32_t nr;                 /* reported links (>= nb: fixed-joint links kept, _model.flatten) */
    const int32_t *clink;       /* [nc] link whose net contact force a candidate adds to */
    /* joint drives (PhysX articulation drives as an implicit spring-damper per
     * substep), NULL = none: kp (q* - q - h qd) + kd (qd* - qd) with h kd + h^2 kp on M's diagonal */
    const double *dkp;          /* [nd] or NULL */
    const double *dkd;          /* [nd] or NULL */
    /* ---- convex hulls and self-collision */
    const int32_t *cdyn;        /* [nc] hull slot (0..3) of a hull's dynamic ground candidate, -1 fixed point */
    const int32_t *shkind;      /* [ns] 0 sphere 1 capsule 2 box 3 cylinder 4 hull */
    const int32_t *shbody;      /* [ns] */
    const int32_t *shlink;      /* [ns] */
    const double *shpose;       /* [ns][12] body frame R (9) t (3) */
    const double *shsize;       /* [ns][3] sphere r | capsule r, half length | box half extents */
    const double *shmargin;     /* [ns] core radius of the pair narrowphase */
    const double *shsphere;     /* [ns][4] bounding sphere, body frame centre + radius */
    const double *hverts;       /* [nhv][4] hull vertices, body frame xyz + core factor */
    const int32_t *shv0, *shv1; /* [ns] hull vertex range */
    int32_t npair;
    const int32_t *pair_a, *pair_b, *pair_kind; /* [npair] shape a < shape b; 0 SS 1 SC 2 CC 3 GJK */
    int32_t npool;              /* self-contact slots per env (pair order, later contacts dropped) */
    int32_t self_collide;       /* filter-0 actor: self-collision pairs enabled */
    const double *pverts;       /* [npv][4] a hull's self-collision core vertices (subset of hverts) */
    const int32_t *shp0, *shp1; /* [ns] their range */
    /* the self-contact departures of DESIGN.md 3.12 as switches, for tools/pool_policy_study.py (0 = the
     * product's rules): bit 0 overlapping cores make a contact (centres' direction, depth = both margins)
     * instead of none; bit 1 every self-contact row responds (no MIN_RESPONSE bound).  The pool cap is npool. */
    int32_t pool_policy;
} OModel;

typedef struct {
    double dt;
    int32_t substeps;
    double gravity[3];
    int32_t pos_iters, vel_iters;
    double contact_offset, rest_offset, max_depen_vel;
    int32_t collect_contacts;
    int32_t has_ground;
    double ground_friction;
    double limit_margin;        /* joint-limit rows active within this distance of a limit */
    /* heightfield-grid triangle mesh: vertex (i,j) at tverts[3*(i*tcols+j)], world
     * coordinates; grid point (i,j) at (tx0 + i*ths, ty0 + j*ths); cell (i,j) -> triangles
     * (v[i,j], v[i+1,j+1], v[i,j+1]), (v[i,j], v[i+1,j], v[i+1,j+1]) */
    int32_t has_terrain;
    int32_t trows, tcols;
    const float *tverts;
    double tx0, ty0, ths;
    double terrain_friction;
    /* physx.solver_type (cfg/config.yaml:31): 0 PGS (the kernels' solver), 1 TGS, 2 TGS with the joint velocity
     * limit applied in each position sub-step -- 1 and 2 oracle only, the study of
     * pos_iters sub-steps of h / pos_iters, each row's separation advanced by the displacement
     * integrated so far, positions integrated with the sub-steps' velocities, no bias in the velocity phase */
    int32_t solver_type;
} OParams;

/* ---------------------------------------------------------------- helpers */
static inline void cross3(const real *a, const real *b, real *o) {
    real x = a[1] * b[2] - a[2] * b[1], y = a[2] * b[0] - a[0] * b[2], z = a[0] * b[1] - a[1] * b[0];
    o[0] = x; o[1] = y; o[2] = z;
}
static inline real dot3(const real *a, const real *b) { return a[0] * b[0] + a[1] * b[1] + a[2] * b[2]; }
static inline void matvec3(const real *R, const real *v, real *o) {
    real x = R[0] * v[0] + R[1] * v[1] + R[2] * v[2];
    real y = R[3] * v[0] + R[4] * v[1] + R[5] * v[2];
    real z = R[6] * v[0] + R[7] * v[1] + R[8] * v[2];
    o[0] = x; o[1] = y; o[2] = z;
}
static inline void matmul3(const real *A, const real *B, real *C) {
    real T[9];
    for (int i = 0; i < 3; ++i)
        for (int j = 0; j < 3; ++j) T[3 * i + j] = A[3 * i] * B[j] + A[3 * i + 1] * B[3 + j] + A[3 * i + 2] * B[6 + j];
    memcpy(C, T, sizeof(T));
}
/* Rodrigues rotation about unit axis a by angle t */
static void axis_angle(const real *a, real t, real *R) {
    real c = cos(t), s = sin(t), C = 1 - c;
    real x = a[0], y = a[1], z = a[2];
    R[0] = c + x * x * C;     R[1] = x * y * C - z * s; R[2] = x * z * C + y * s;
    R[3] = y * x * C + z * s; R[4] = c + y * y * C;     R[5] = y * z * C - x * s;
    R[6] = z * x * C - y * s; R[7] = z * y * C + x * s; R[8] = c + z * z * C;
}
static void quat_to_mat(const real *q, real *R) { /* xyzw */
    real x = q[0], y = q[1], z = q[2], w = q[3];
    R[0] = 1 - 2 * (y * y + z * z); R[1] = 2 * (x * y - z * w);     R[2] = 2 * (x * z + y * w);
    R[3] = 2 * (x * y + z * w);     R[4] = 1 - 2 * (x * x + z * z); R[5] = 2 * (y * z - x * w);
    R[6] = 2 * (x * z - y * w);     R[7] = 2 * (y * z + x * w);     R[8] = 1 - 2 * (x * x + y * y);
}

/* ---------------------------------------------------------------- terrain mesh
 * Sphere vs triangle, stated with a plane projection and edge clamping (the kernel walks the
 * Voronoi regions instead): the projection of c inside the triangle -> face contact along the face
 * normal (also from behind, up to r + TERRAIN_BACK); otherwise the nearest point of the three
 * edges, from the front side only; triangles facing down (n_z < TERRAIN_DOWN_NZ, inverted by the
 * slope-threshold vertex moves) are skipped.  The triangle CLOSEST to the centre gives the contact (first
 * found on ties, visiting the cell under the centre first, then every cell in (i, j) order).  Full scan of a
 * window 3 cells wider than any triangle of a grid cell can reach (vertices move at most one cell). */
#define TERRAIN_BACK 0.1
#define TERRAIN_DOWN_NZ (-0.5) /* downward-facing (inverted) triangles generate no contact */
static void seg_closest(const real *p, const real *a, const real *b, real *q) {
    real ab[3] = {b[0] - a[0], b[1] - a[1], b[2] - a[2]}, ap[3] = {p[0] - a[0], p[1] - a[1], p[2] - a[2]};
    const real l2 = dot3(ab, ab);
    real t = l2 > 0 ? dot3(ap, ab) / l2 : 0;
    if (t < 0) t = 0;
    if (t > 1) t = 1;
    for (int k = 0; k < 3; ++k) q[k] = a[k] + t * ab[k];
}
/* candidate surface of one triangle: key = distance from the centre to the triangle (the closest
 * surface wins), separation signed (negative behind a face) */
static void tri_test(const real *p, real r, real thr, const real *a, const real *b, const real *c, real *bkey,
                     real *bsep, real *n) {
    real e1[3] = {b[0] - a[0], b[1] - a[1], b[2] - a[2]}, e2[3] = {c[0] - a[0], c[1] - a[1], c[2] - a[2]}, nf[3];
    cross3(e1, e2, nf);
    const real l = sqrt(dot3(nf, nf));
    if (!(l * l > 1e-14)) return;
    for (int k = 0; k < 3; ++k) nf[k] /= l;
    if (nf[2] < TERRAIN_DOWN_NZ) return;
    const real ap[3] = {p[0] - a[0], p[1] - a[1], p[2] - a[2]};
    const real sd = dot3(nf, ap);
    if (sd > thr || sd < -(r + TERRAIN_BACK)) return;
    /* barycentric coordinates of the projection */
    const real proj[3] = {p[0] - sd * nf[0], p[1] - sd * nf[1], p[2] - sd * nf[2]};
    const real v0[3] = {proj[0] - a[0], proj[1] - a[1], proj[2] - a[2]};
    const real d00 = dot3(e1, e1), d01 = dot3(e1, e2), d11 = dot3(e2, e2), d20 = dot3(v0, e1), d21 = dot3(v0, e2);
    const real den = d00 * d11 - d01 * d01;
    const real bv = (d11 * d20 - d01 * d21) / den, bw = (d00 * d21 - d01 * d20) / den;
    if (bv >= 0 && bw >= 0 && bv + bw <= 1) {
        const real key = fabs(sd);
        if (key < *bkey) { *bkey = key; *bsep = sd - r; n[0] = nf[0]; n[1] = nf[1]; n[2] = nf[2]; }
        return;
    }
    if (sd < 0) return;
    real q[3], qq[3], dbest = 1e300;
    const real *ends[3][2] = {{a, b}, {b, c}, {c, a}};
    for (int k = 0; k < 3; ++k) {
        seg_closest(p, ends[k][0], ends[k][1], qq);
        const real d2 = (p[0] - qq[0]) * (p[0] - qq[0]) + (p[1] - qq[1]) * (p[1] - qq[1]) + (p[2] - qq[2]) * (p[2] - qq[2]);
        if (d2 < dbest) { dbest = d2; q[0] = qq[0]; q[1] = qq[1]; q[2] = qq[2]; }
    }
    if (dbest > thr * thr) return;
    const real dist = sqrt(dbest);
    if (dist < *bkey) {
        *bkey = dist;
        *bsep = dist - r;
        if (dist > 1e-7) { for (int k = 0; k < 3; ++k) n[k] = (p[k] - q[k]) / dist; }
        else { n[0] = nf[0]; n[1] = nf[1]; n[2] = nf[2]; }
    }
}
static int terrain_query(const OParams *pp, const real *p, real r, real thr, real *sep, real *n) {
    const real hs = (real)pp->ths;
    const int gi = (int)floor((p[0] - (real)pp->tx0) / hs), gj = (int)floor((p[1] - (real)pp->ty0) / hs);
    const real reach = thr > r + TERRAIN_BACK ? thr : r + TERRAIN_BACK;
    const int w = (int)ceil(reach / hs) + 3;
    real bkey = 1e300, best = 1e300;
    const int centre = gi >= 0 && gi <= pp->trows - 2 && gj >= 0 && gj <= pp->tcols - 2;
    for (int pass = centre ? 0 : 1; pass < 2; ++pass)
    for (int i = pass ? gi - w : gi; i <= (pass ? gi + w : gi); ++i) {
        if (i < 0 || i > pp->trows - 2) continue;
        for (int j = pass ? gj - w : gj; j <= (pass ? gj + w : gj); ++j) {
            if (j < 0 || j > pp->tcols - 2) continue;
            if (pass && centre && i == gi && j == gj) continue;
            real v[4][3];
            const int64_t id[4] = {(int64_t)i * pp->tcols + j, (int64_t)i * pp->tcols + j + 1,
                                   (int64_t)(i + 1) * pp->tcols + j, (int64_t)(i + 1) * pp->tcols + j + 1};
            for (int k = 0; k < 4; ++k)
                for (int a = 0; a < 3; ++a) v[k][a] = (real)pp->tverts[3 * id[k] + a];
            tri_test(p, r, thr, v[0], v[3], v[1], &bkey, &best, n);
            tri_test(p, r, thr, v[0], v[2], v[3], &bkey, &best, n);
        }
    }
    if (!(best < thr - r)) return 0;
    *sep = best;
    return 1;
}
/* contact frame tangents: world x projected on the contact plane (world y when n ~ x), t2 = n x t1 */
static void tangents(const real *n, real *t1, real *t2) {
    real a[3] = {1 - n[0] * n[0], -n[0] * n[1], -n[0] * n[2]};
    real l2 = dot3(a, a);
    if (l2 < 1e-6) { a[0] = -n[1] * n[0]; a[1] = 1 - n[1] * n[1]; a[2] = -n[1] * n[2]; l2 = dot3(a, a); }
    const real l = sqrt(l2);
    for (int k = 0; k < 3; ++k) t1[k] = a[k] / l;
    cross3(n, t1, t2);
}

/* ---------------------------------------------------------------- convex hull vs ground
 * Vertices of hull shape sh whose height is below contact_offset, reduced to at most 4 contact points:
 * the deepest; the one farthest from it horizontally; the one spanning the largest horizontal triangle with
 * those two; the one farthest outside that triangle.  First vertex index wins ties; a step whose best
 * value is <= 1e-10 ends the selection. */
static int hull_ground_select(const OModel *m, int sh, const real *R, const real *P, real rootz, real off,
                              int *sel) {
    const int v0 = m->shv0[sh], v1 = m->shv1[sh];
    int n = 0, i0 = -1;
    real zmin = 1e300;
#define HV(k, out)                                                           \
    {                                                                        \
        real vl[3] = {(real)m->hverts[4 * (k)], (real)m->hverts[4 * (k) + 1], (real)m->hverts[4 * (k) + 2]}; \
        matvec3(R, vl, out);                                                 \
        for (int a_ = 0; a_ < 3; ++a_) out[a_] += P[a_];                     \
        out[2] += rootz;                                                     \
    }
    for (int k = v0; k < v1; ++k) { real w[3]; HV(k, w); if (w[2] < zmin) { zmin = w[2]; i0 = k; } }
    if (i0 < 0 || !(zmin < off)) return 0;
    real p0[3]; HV(i0, p0);
    sel[n++] = i0;
    int i1 = -1; real best = 1e-10;
    for (int k = v0; k < v1; ++k) {
        real w[3]; HV(k, w);
        if (!(w[2] < off)) continue;
        const real d2 = (w[0] - p0[0]) * (w[0] - p0[0]) + (w[1] - p0[1]) * (w[1] - p0[1]);
        if (d2 > best) { best = d2; i1 = k; }
    }
    if (i1 < 0) return n;
    real p1[3]; HV(i1, p1);
    sel[n++] = i1;
    const real ex = p1[0] - p0[0], ey = p1[1] - p0[1];
    int i2 = -1; best = 1e-10;
    for (int k = v0; k < v1; ++k) {
        real w[3]; HV(k, w);
        if (!(w[2] < off)) continue;
        const real a = fabs(ex * (w[1] - p0[1]) - ey * (w[0] - p0[0]));
        if (a > best) { best = a; i2 = k; }
    }
    if (i2 < 0) return n;
    real p2[3]; HV(i2, p2);
    sel[n++] = i2;
    const real sg = (ex * (p2[1] - p0[1]) - ey * (p2[0] - p0[0])) > 0 ? 1 : -1;
    int i3 = -1; best = 1e-10;
    for (int k = v0; k < v1; ++k) {
        real w[3]; HV(k, w);
        if (!(w[2] < off)) continue;
        const real e0 = sg * ((p1[0] - p0[0]) * (w[1] - p0[1]) - (p1[1] - p0[1]) * (w[0] - p0[0]));
        const real e1 = sg * ((p2[0] - p1[0]) * (w[1] - p1[1]) - (p2[1] - p1[1]) * (w[0] - p1[0]));
        const real e2 = sg * ((p0[0] - p2[0]) * (w[1] - p2[1]) - (p0[1] - p2[1]) * (w[0] - p2[0]));
        real mn = e0 < e1 ? e0 : e1;
        mn = mn < e2 ? mn : e2;
        if (-mn > best) { best = -mn; i3 = k; }
    }
#undef HV
    if (i3 >= 0) sel[n++] = i3;
    return n;
}

/* ---------------------------------------------------------------- self-collision */
typedef struct { real R[9], c[3], sc[3]; } ShapeW; /* world (root-origin-relative) pose + bounding-sphere centre */

/* core support point of shape sh (pose W) in direction d */
static void core_support(const OModel *m, int sh, const ShapeW *W, const real *Rb, const real *Pb, const real *d,
                         real *out) {
    const int kind = m->shkind[sh];
    const double *sz = m->shsize + 3 * sh;
    if (kind == 0) { for (int k = 0; k < 3; ++k) out[k] = W->c[k]; return; }
    if (kind == 1) {
        const real ax[3] = {W->R[2], W->R[5], W->R[8]};
        const real s = dot3(ax, d) >= 0 ? sz[1] : -sz[1];
        for (int k = 0; k < 3; ++k) out[k] = W->c[k] + s * ax[k];
        return;
    }
    if (kind == 3) { /* flat-ended cylinder: rim point of the end disc (core radius r - m, half length h - m) */
        const real mg = (real)m->shmargin[sh];
        const real ax[3] = {W->R[2], W->R[5], W->R[8]};
        const real da = dot3(ax, d);
        real pp[3] = {d[0] - da * ax[0], d[1] - da * ax[1], d[2] - da * ax[2]};
        /* projected once more (d nearly along the axis: the subtraction cancels; gs_pairs.h core_support) */
        const real pa = dot3(ax, pp);
        for (int k = 0; k < 3; ++k) pp[k] -= pa * ax[k];
        const real lp = sqrt(dot3(pp, pp));
        const real s = da >= 0 ? sz[1] - mg : -(sz[1] - mg);
        for (int k = 0; k < 3; ++k) out[k] = W->c[k] + s * ax[k] + (lp > 1e-12 ? (sz[0] - mg) * pp[k] / lp : 0);
        return;
    }
    if (kind == 2) {
        const real mg = (real)m->shmargin[sh];
        for (int k = 0; k < 3; ++k) out[k] = W->c[k];
        for (int i = 0; i < 3; ++i) {
            const real e[3] = {W->R[i], W->R[3 + i], W->R[6 + i]};
            const real s = dot3(e, d) >= 0 ? sz[i] - mg : -(sz[i] - mg);
            for (int k = 0; k < 3; ++k) out[k] += s * e[k];
        }
        return;
    }
    /* hull: body-frame vertices moved toward the centroid by the margin */
    real dl[3] = {Rb[0] * d[0] + Rb[3] * d[1] + Rb[6] * d[2], Rb[1] * d[0] + Rb[4] * d[1] + Rb[7] * d[2],
                  Rb[2] * d[0] + Rb[5] * d[1] + Rb[8] * d[2]};
    const double *cc = m->shsphere + 4 * sh;
    real best = -1e300, bv[3] = {0, 0, 0};
    for (int k = m->shp0[sh]; k < m->shp1[sh]; ++k) {
        const double *v = m->pverts + 4 * k;
        const real f = (real)v[3];
        const real p[3] = {cc[0] + f * (v[0] - cc[0]), cc[1] + f * (v[1] - cc[1]), cc[2] + f * (v[2] - cc[2])};
        const real t = dot3(p, dl);
        if (t > best) { best = t; bv[0] = p[0]; bv[1] = p[1]; bv[2] = p[2]; }
    }
    matvec3(Rb, bv, out);
    for (int k = 0; k < 3; ++k) out[k] += Pb[k];
}

/* Centroid of shape sh's core support feature in direction d: the core points within FEATURE_EPS of the
 * support plane (box corners, hull vertices; a cylinder's end disc, side line or rim point; a capsule's
 * segment or end; a sphere's centre).  Returns the feature's extent (largest distance of its points from the
 * centroid), 0 for a single point. */
#define FEATURE_EPS 2e-3
static real core_feature(const OModel *m, int sh, const ShapeW *W, const real *Rb, const real *Pb, const real *d,
                         real *cen) {
    const int kind = m->shkind[sh];
    const double *sz = m->shsize + 3 * sh;
    const real mg = (real)m->shmargin[sh];
    if (kind == 0) { for (int k = 0; k < 3; ++k) cen[k] = W->c[k]; return 0; }
    if (kind == 1 || kind == 3) {
        const real ax[3] = {W->R[2], W->R[5], W->R[8]};
        const real hl = kind == 1 ? (real)sz[1] : (real)sz[1] - mg, rr = kind == 1 ? 0 : (real)sz[0] - mg;
        const real da = dot3(ax, d);
        real pp[3] = {d[0] - da * ax[0], d[1] - da * ax[1], d[2] - da * ax[2]};
        const real lp = sqrt(dot3(pp, pp));
        /* the two ends' support heights differ by 2 hl |da|: both ends within the band -> the side segment */
        const int side = 2 * hl * fabs(da) <= FEATURE_EPS;
        /* a cylinder end disc faces d when the rim spread 2 rr lp stays within the band */
        const int disc = kind == 3 && 2 * rr * lp <= FEATURE_EPS;
        const real s = side ? 0 : (da >= 0 ? hl : -hl);
        for (int k = 0; k < 3; ++k) cen[k] = W->c[k] + s * ax[k] + (disc || !(lp > 1e-12) ? 0 : rr * pp[k] / lp);
        return side ? hl : (disc ? rr : 0);
    }
    if (kind == 2) {
        real hmax = -1e300, pts[8][3];
        for (int c = 0; c < 8; ++c) {
            for (int k = 0; k < 3; ++k) pts[c][k] = W->c[k];
            for (int i = 0; i < 3; ++i) {
                const real sg = (c >> i & 1) ? 1 : -1;
                for (int k = 0; k < 3; ++k) pts[c][k] += sg * ((real)sz[i] - mg) * W->R[3 * k + i];
            }
            const real h = dot3(pts[c], d);
            if (h > hmax) hmax = h;
        }
        int n = 0;
        for (int k = 0; k < 3; ++k) cen[k] = 0;
        for (int c = 0; c < 8; ++c)
            if (dot3(pts[c], d) >= hmax - FEATURE_EPS) { for (int k = 0; k < 3; ++k) cen[k] += pts[c][k]; ++n; }
        for (int k = 0; k < 3; ++k) cen[k] /= n;
        real ext = 0;
        for (int c = 0; c < 8; ++c)
            if (dot3(pts[c], d) >= hmax - FEATURE_EPS) {
                const real dd[3] = {pts[c][0] - cen[0], pts[c][1] - cen[1], pts[c][2] - cen[2]};
                const real l = sqrt(dot3(dd, dd));
                if (l > ext) ext = l;
            }
        return ext;
    }
    /* hull (body-frame core vertices) */
    const real dl[3] = {Rb[0] * d[0] + Rb[3] * d[1] + Rb[6] * d[2], Rb[1] * d[0] + Rb[4] * d[1] + Rb[7] * d[2],
                        Rb[2] * d[0] + Rb[5] * d[1] + Rb[8] * d[2]};
    const double *cc = m->shsphere + 4 * sh;
    real hmax = -1e300;
    for (int k = m->shp0[sh]; k < m->shp1[sh]; ++k) {
        const double *v = m->pverts + 4 * k;
        const real f = (real)v[3];
        const real p[3] = {cc[0] + f * (v[0] - cc[0]), cc[1] + f * (v[1] - cc[1]), cc[2] + f * (v[2] - cc[2])};
        const real h = dot3(p, dl);
        if (h > hmax) hmax = h;
    }
    real acc[3] = {0, 0, 0};
    int n = 0;
    for (int k = m->shp0[sh]; k < m->shp1[sh]; ++k) {
        const double *v = m->pverts + 4 * k;
        const real f = (real)v[3];
        const real p[3] = {cc[0] + f * (v[0] - cc[0]), cc[1] + f * (v[1] - cc[1]), cc[2] + f * (v[2] - cc[2])};
        if (dot3(p, dl) >= hmax - FEATURE_EPS) { for (int t = 0; t < 3; ++t) acc[t] += p[t]; ++n; }
    }
    for (int t = 0; t < 3; ++t) acc[t] /= n;
    real ext = 0;
    for (int k = m->shp0[sh]; k < m->shp1[sh]; ++k) {
        const double *v = m->pverts + 4 * k;
        const real f = (real)v[3];
        const real p[3] = {cc[0] + f * (v[0] - cc[0]), cc[1] + f * (v[1] - cc[1]), cc[2] + f * (v[2] - cc[2])};
        if (dot3(p, dl) >= hmax - FEATURE_EPS) {
            const real dd[3] = {p[0] - acc[0], p[1] - acc[1], p[2] - acc[2]};
            const real l = sqrt(dot3(dd, dd));
            if (l > ext) ext = l;
        }
    }
    matvec3(Rb, acc, cen);
    for (int t = 0; t < 3; ++t) cen[t] += Pb[t];
    return ext;
}

/* closest point of conv(W[0..k)) to the origin: every vertex subset whose affine closest point has positive
 * barycentrics is a candidate, the nearest wins (first subset on ties); returns the subset mask */
static int simplex_closest(real W[4][3], int k, real *v, real *lam) {
    real best = 1e300;
    int bm = 0;
    for (int mask = 1; mask < (1 << k); ++mask) {
        int id[4], n = 0;
        for (int i = 0; i < k; ++i) if (mask >> i & 1) id[n++] = i;
        real l[4] = {1, 0, 0, 0}, p[3];
        if (n == 1) {
            for (int a = 0; a < 3; ++a) p[a] = W[id[0]][a];
        } else {
            real E[3][3], G[3][3] = {{0, 0, 0}, {0, 0, 0}, {0, 0, 0}}, r[3], mu[3];
            for (int j = 1; j < n; ++j) for (int a = 0; a < 3; ++a) E[j - 1][a] = W[id[j]][a] - W[id[0]][a];
            const int q = n - 1;
            for (int i = 0; i < q; ++i) {
                r[i] = -dot3(W[id[0]], E[i]);
                for (int j = 0; j < q; ++j) G[i][j] = dot3(E[i], E[j]);
            }
            if (q == 1) {
                if (!(G[0][0] > 1e-18)) continue;
                mu[0] = r[0] / G[0][0];
            } else if (q == 2) {
                const real det = G[0][0] * G[1][1] - G[0][1] * G[1][0];
                if (!(fabs(det) > 1e-12 * G[0][0] * G[1][1]) || !(det != 0)) continue;
                mu[0] = (r[0] * G[1][1] - G[0][1] * r[1]) / det;
                mu[1] = (G[0][0] * r[1] - r[0] * G[1][0]) / det;
            } else {
                const real det = G[0][0] * (G[1][1] * G[2][2] - G[1][2] * G[2][1]) -
                                 G[0][1] * (G[1][0] * G[2][2] - G[1][2] * G[2][0]) +
                                 G[0][2] * (G[1][0] * G[2][1] - G[1][1] * G[2][0]);
                if (!(fabs(det) > 1e-12 * G[0][0] * G[1][1] * G[2][2]) || !(det != 0)) continue;
                for (int c = 0; c < 3; ++c) {
                    real Gc[3][3];
                    for (int i = 0; i < 3; ++i) for (int j = 0; j < 3; ++j) Gc[i][j] = j == c ? r[i] : G[i][j];
                    mu[c] = (Gc[0][0] * (Gc[1][1] * Gc[2][2] - Gc[1][2] * Gc[2][1]) -
                             Gc[0][1] * (Gc[1][0] * Gc[2][2] - Gc[1][2] * Gc[2][0]) +
                             Gc[0][2] * (Gc[1][0] * Gc[2][1] - Gc[1][1] * Gc[2][0])) / det;
                }
            }
            real l0 = 1;
            int ok = 1;
            for (int j = 0; j < q; ++j) { l0 -= mu[j]; l[j + 1] = mu[j]; if (!(mu[j] > 1e-12)) ok = 0; }
            l[0] = l0;
            if (!ok || !(l0 > 1e-12)) continue;
            for (int a = 0; a < 3; ++a) {
                p[a] = W[id[0]][a];
                for (int j = 0; j < q; ++j) p[a] += mu[j] * E[j][a];
            }
        }
        const real d2 = dot3(p, p);
        if (d2 < best) {
            best = d2;
            bm = mask;
            for (int a = 0; a < 3; ++a) v[a] = p[a];
            for (int i = 0, j = 0; i < k; ++i) lam[i] = (mask >> i & 1) ? l[j++] : 0;
        }
    }
    return bm;
}

/* GJK distance between the cores of shapes a and b: closest points pa, pb, separating vector vout (the final
 * simplex's closest point, = pa - pb); returns the distance, 0 when the cores overlap */
/* narrowphase workload counters (analysis only: oracle_pair_stats, tools/pool_overflow_study.py): pairs tested,
 * bounding spheres met, GJK calls, GJK iterations, contacts kept, deep core overlaps skipped (GS_DEEP_SKIP),
 * contacts dropped at the pool cap (not thread-safe: read them from single-threaded runs) */
static long long g_pair_stats[7];

static real gjk_cores(const OModel *m, int sa, int sb, const ShapeW *Wa, const ShapeW *Wb, const real *Ra,
                      const real *Pa, const real *Rb, const real *Pb, real *pa, real *pb, real *vout) {
    ++g_pair_stats[2];
    real v[3] = {Wa->sc[0] - Wb->sc[0], Wa->sc[1] - Wb->sc[1], Wa->sc[2] - Wb->sc[2]};
    if (dot3(v, v) < 1e-18) { v[0] = 1; v[1] = 0; v[2] = 0; }
    real W[4][3], A[4][3], B[4][3], lam[4] = {1, 0, 0, 0};
    int k = 0;
    int sepd = 0; /* a support plane with v.w > 1e-4 vv certified a positive distance (gs_pairs.h gjk_cores) */
    for (int it = 0; it < 32; ++it) {
        const real nv[3] = {-v[0], -v[1], -v[2]};
        real a[3], b[3], w[3];
        ++g_pair_stats[3];
        core_support(m, sa, Wa, Ra, Pa, nv, a);
        core_support(m, sb, Wb, Rb, Pb, v, b);
        for (int t = 0; t < 3; ++t) w[t] = a[t] - b[t];
        const real vv = dot3(v, v);
#ifdef ORACLE_GJK_TRACE  /* debug builds only */
        fprintf(stderr, "ogjk %d-%d it %d k %d v %.9g %.9g %.9g w %.9g %.9g %.9g vv %.9g vw %.9g\n", sa, sb, it, k,
                (double)v[0], (double)v[1], (double)v[2], (double)w[0], (double)w[1], (double)w[2], (double)vv,
                (double)dot3(v, w));
#endif
        if (dot3(v, w) > (real)1e-4 * vv) sepd = 1;
        if (k > 0 && vv - dot3(v, w) <= (real)GJK_TOL * vv + (real)1e-14) break;
        /* a step along the segment from the closest point of the first kold simplex points (a point of the
         * Minkowski difference, witnesses the same combination of A and B) to w; the simplex becomes {that point,
         * w}; 0 when rounding leaves no progress (the simplex cut back to kold points) -- gs_pairs.h gjk_cores */
        int step = -1; /* -1: none; otherwise kold */
        int dup = 0;
        for (int i = 0; i < k; ++i) {
            const real d[3] = {W[i][0] - w[0], W[i][1] - w[1], W[i][2] - w[2]};
            if (dot3(d, d) < 1e-16) dup = 1;
        }
        /* a repeated support point before convergence: v is off by the subset solve's rounding */
        if (dup) step = k;
        int mask = 0;
        real l4[4];
        if (step < 0) {
            for (int t = 0; t < 3; ++t) { W[k][t] = w[t]; A[k][t] = a[t]; B[k][t] = b[t]; }
            ++k;
            mask = simplex_closest(W, k, v, l4);
            if (!mask && !sepd) return 0;
            /* rounding rejected every subset with the new support point w although w lies beyond the old closest
             * point's support plane, or read the origin as enclosed after a positive distance was certified */
            if (!(mask >> (k - 1) & 1) || (sepd && (mask == 15 || !(dot3(v, v) >= 1e-18)))) step = k - 1;
        }
        if (step >= 0) {
            real Av[3] = {0, 0, 0}, Bv[3] = {0, 0, 0};
            for (int i = 0; i < step; ++i)
                for (int t = 0; t < 3; ++t) { Av[t] += lam[i] * A[i][t]; Bv[t] += lam[i] * B[i][t]; }
            const real Wv[3] = {Av[0] - Bv[0], Av[1] - Bv[1], Av[2] - Bv[2]};
            const real d[3] = {w[0] - Wv[0], w[1] - Wv[1], w[2] - Wv[2]};
            const real dd = dot3(d, d);
            real t = dd > 0 ? -dot3(Wv, d) / dd : 0;
            t = t > 1 ? 1 : t;
            if (!(t > 0)) {
                k = step;
                for (int s = 0; s < 3; ++s) v[s] = Wv[s];
                break;
            }
            for (int s = 0; s < 3; ++s) {
                W[0][s] = Wv[s]; A[0][s] = Av[s]; B[0][s] = Bv[s];
                W[1][s] = w[s]; A[1][s] = a[s]; B[1][s] = b[s];
                v[s] = Wv[s] + t * d[s];
            }
            lam[0] = 1 - t; lam[1] = t; lam[2] = 0; lam[3] = 0;
            k = 2;
            continue;
        }
        int n = 0;
        for (int i = 0; i < k; ++i)
            if (mask >> i & 1) {
                for (int t = 0; t < 3; ++t) { W[n][t] = W[i][t]; A[n][t] = A[i][t]; B[n][t] = B[i][t]; }
                lam[n++] = l4[i];
            }
        k = n;
        if (k == 4 || dot3(v, v) < 1e-18) return 0;
    }
    for (int t = 0; t < 3; ++t) { pa[t] = 0; pb[t] = 0; }
    for (int i = 0; i < k; ++i)
        for (int t = 0; t < 3; ++t) { pa[t] += lam[i] * A[i][t]; pb[t] += lam[i] * B[i][t]; }
    /* the separating direction refined from the final simplex's geometry (the segment's perpendicular, the
     * triangle's plane normal: the same direction as v in exact arithmetic; gs_pairs.h gjk_cores, where float
     * needs it), only from a well-conditioned simplex and within a small angle of v */
    real vr[3] = {v[0], v[1], v[2]};
    if (k == 2 || k == 3) {
        real E0[3], E1[3], pr[3];
        for (int t = 0; t < 3; ++t) { E0[t] = W[1][t] - W[0][t]; E1[t] = W[2][t] - W[0][t]; }
        int ok;
        if (k == 2) {
            const real ee = dot3(E0, E0);
            real c1[3];
            cross3(E0, W[0], c1);
            cross3(c1, E0, pr);
            ok = ee > 0;
            for (int t = 0; t < 3; ++t) pr[t] = ok ? pr[t] / ee : 0;
        } else {
            real nr[3];
            cross3(E0, E1, nr);
            const real nn2 = dot3(nr, nr);
            ok = nn2 > 1e-8 * dot3(E0, E0) * dot3(E1, E1);
            const real s = ok ? dot3(nr, W[0]) / nn2 : 0;
            for (int t = 0; t < 3; ++t) pr[t] = s * nr[t];
        }
        const real vv = dot3(v, v), pp = dot3(pr, pr), vp = dot3(v, pr);
        if (ok && vp > 0 && vp * vp >= 0.9999 * vv * pp) for (int t = 0; t < 3; ++t) vr[t] = pr[t];
    }
    for (int t = 0; t < 3; ++t) vout[t] = vr[t];
    return sqrt(dot3(v, v));
}

/* closest points of segments p1q1, p2q2 (Ericson): parameters s, t; returns a e - b^2 and a, e */
static void seg_seg(const real *p1, const real *q1, const real *p2, const real *q2, real *s_, real *t_, real *den_,
                    real *a_, real *e_) {
    real d1[3], d2[3], r[3];
    for (int k = 0; k < 3; ++k) { d1[k] = q1[k] - p1[k]; d2[k] = q2[k] - p2[k]; r[k] = p1[k] - p2[k]; }
    const real a = dot3(d1, d1), e = dot3(d2, d2), f = dot3(d2, r);
    real s = 0, t = 0, den = 0;
    if (a <= 1e-12 && e <= 1e-12) { s = t = 0; }
    else if (a <= 1e-12) { s = 0; t = f / e; t = t < 0 ? 0 : (t > 1 ? 1 : t); }
    else {
        const real c = dot3(d1, r);
        if (e <= 1e-12) { t = 0; s = -c / a; s = s < 0 ? 0 : (s > 1 ? 1 : s); }
        else {
            const real b = dot3(d1, d2);
            den = a * e - b * b;
            if (den > 0) { s = (b * f - c * e) / den; s = s < 0 ? 0 : (s > 1 ? 1 : s); }
            else s = 0;
            t = (b * s + f) / e;
            if (t < 0) { t = 0; s = -c / a; s = s < 0 ? 0 : (s > 1 ? 1 : s); }
            else if (t > 1) { t = 1; s = (b - c) / a; s = s < 0 ? 0 : (s > 1 ? 1 : s); }
        }
    }
    *s_ = s; *t_ = t; *den_ = den; *a_ = a; *e_ = e;
}

typedef struct { real x[3], n[3], sep, mu; int ba, bb, la, lb; } PairContact;

/* self-contacts of one env, pair order, at most npool: broadphase on the shapes' bounding spheres
 * (within contact_offset), closed-form sphere / capsule pairs, GJK on margin-rounded cores otherwise */
static int self_contacts(const OModel *m, const OParams *p, real R[][9], real P[][3], const real *mu_shape,
                         PairContact *out) {
    ShapeW W[64];
    const real off = (real)p->contact_offset;
    for (int sh = 0; sh < m->ns; ++sh) {
        const int b = m->shbody[sh];
        real Rl[9], tl[3], t[3], sc[3];
        for (int k = 0; k < 9; ++k) Rl[k] = (real)m->shpose[12 * sh + k];
        for (int k = 0; k < 3; ++k) { tl[k] = (real)m->shpose[12 * sh + 9 + k]; sc[k] = (real)m->shsphere[4 * sh + k]; }
        matmul3(R[b], Rl, W[sh].R);
        matvec3(R[b], tl, t);
        for (int k = 0; k < 3; ++k) W[sh].c[k] = P[b][k] + t[k];
        matvec3(R[b], sc, t);
        for (int k = 0; k < 3; ++k) W[sh].sc[k] = P[b][k] + t[k];
    }
    int n = 0;
    for (int q = 0; q < m->npair && n < m->npool; ++q) {
        const int a = m->pair_a[q], b = m->pair_b[q], kind = m->pair_kind[q];
        const real d[3] = {W[a].sc[0] - W[b].sc[0], W[a].sc[1] - W[b].sc[1], W[a].sc[2] - W[b].sc[2]};
        const real rr = (real)m->shsphere[4 * a + 3] + (real)m->shsphere[4 * b + 3] + off;
        ++g_pair_stats[0];
        if (!(dot3(d, d) < rr * rr)) continue;
        ++g_pair_stats[1];
        const int ba = m->shbody[a], bb = m->shbody[b];
        const real ra = (real)m->shmargin[a], rb = (real)m->shmargin[b];
        real pa[2][3], pb[2][3];
        int nct = 1, gdeep = 0, gnorm = 0;
        real gn[3] = {0, 0, 1}, gdist = 0; /* GJK pairs: the contact normal and the cores' distance */
        if (kind == 0) {
            for (int k = 0; k < 3; ++k) { pa[0][k] = W[a].c[k]; pb[0][k] = W[b].c[k]; }
        } else if (kind == 1) {
            const int sa_sph = m->shkind[a] == 0;
            const int cap = sa_sph ? b : a, sph = sa_sph ? a : b;
            const real ax[3] = {W[cap].R[2], W[cap].R[5], W[cap].R[8]}, hl = (real)m->shsize[3 * cap + 1];
            real e0[3], e1[3], q3[3];
            for (int k = 0; k < 3; ++k) { e0[k] = W[cap].c[k] - hl * ax[k]; e1[k] = W[cap].c[k] + hl * ax[k]; }
            seg_closest(W[sph].c, e0, e1, q3);
            for (int k = 0; k < 3; ++k) {
                (sa_sph ? pa : pb)[0][k] = W[sph].c[k];
                (sa_sph ? pb : pa)[0][k] = q3[k];
            }
        } else if (kind == 2) {
            const real axa[3] = {W[a].R[2], W[a].R[5], W[a].R[8]}, axb[3] = {W[b].R[2], W[b].R[5], W[b].R[8]};
            const real ha = (real)m->shsize[3 * a + 1], hb = (real)m->shsize[3 * b + 1];
            real p1[3], q1[3], p2[3], q2[3];
            for (int k = 0; k < 3; ++k) {
                p1[k] = W[a].c[k] - ha * axa[k]; q1[k] = W[a].c[k] + ha * axa[k];
                p2[k] = W[b].c[k] - hb * axb[k]; q2[k] = W[b].c[k] + hb * axb[k];
            }
            real s, t, den, aa, ee;
            seg_seg(p1, q1, p2, q2, &s, &t, &den, &aa, &ee);
            int two = 0;
            real lo = 0, hi = 0;
            if (aa > 1e-12 && ee > 1e-12 && den <= 1e-4 * aa * ee) {
                /* parallel: both ends of the overlap of B's projection onto A */
                real d1[3], w0[3], w1[3];
                for (int k = 0; k < 3; ++k) { d1[k] = q1[k] - p1[k]; w0[k] = p2[k] - p1[k]; w1[k] = q2[k] - p1[k]; }
                const real s0 = dot3(w0, d1) / aa, s1 = dot3(w1, d1) / aa;
                lo = s0 < s1 ? s0 : s1; hi = s0 < s1 ? s1 : s0;
                lo = lo < 0 ? 0 : lo; hi = hi > 1 ? 1 : hi;
                two = hi - lo > 1e-3;
            }
            if (two) {
                nct = 2;
                for (int c = 0; c < 2; ++c) {
                    const real sc2 = c == 0 ? lo : hi;
                    for (int k = 0; k < 3; ++k) pa[c][k] = p1[k] + sc2 * (q1[k] - p1[k]);
                    seg_closest(pa[c], p2, q2, pb[c]);
                }
            } else {
                for (int k = 0; k < 3; ++k) { pa[0][k] = p1[k] + s * (q1[k] - p1[k]); pb[0][k] = p2[k] + t * (q2[k] - p2[k]); }
            }
        } else {
            real vg[3];
            const real dist = gjk_cores(m, a, b, &W[a], &W[b], R[ba], P[ba], R[bb], P[bb], pa[0], pb[0], vg);
            if (!(dist > 1e-9)) { /* overlapping cores: centres' direction, depth = both margins */
                gdeep = 1;
                for (int k = 0; k < 3; ++k) { pa[0][k] = W[a].sc[k]; pb[0][k] = W[b].sc[k]; }
            } else {
                /* the contact point: the centroid of the smaller of the two support features facing each
                 * other (a face's, not GJK's arbitrary point of it), kept at the cores' distance */
                const real nn[3] = {vg[0] / dist, vg[1] / dist, vg[2] / dist};
                gnorm = 1; gdist = dist;
                for (int k = 0; k < 3; ++k) gn[k] = nn[k];
                const real mn[3] = {-nn[0], -nn[1], -nn[2]};
                real ca[3], cb[3];
                const real ea = core_feature(m, a, &W[a], R[ba], P[ba], mn, ca);
                const real eb = core_feature(m, b, &W[b], R[bb], P[bb], nn, cb);
                for (int k = 0; k < 3; ++k) {
                    if (ea <= eb) { pa[0][k] = ca[k]; pb[0][k] = ca[k] - dist * nn[k]; }
                    else { pb[0][k] = cb[k]; pa[0][k] = cb[k] + dist * nn[k]; }
                }
            }
        }
        for (int c = 0; c < nct && n < m->npool; ++c) {
            real nn[3] = {pa[c][0] - pb[c][0], pa[c][1] - pb[c][1], pa[c][2] - pb[c][2]};
            real dist = sqrt(dot3(nn, nn));
            const int deep = gdeep;
            if (gnorm) {
                for (int k = 0; k < 3; ++k) nn[k] = gn[k];
                dist = gdist;
            } else if (!(dist > 1e-9)) {
                real f[3] = {W[a].sc[0] - W[b].sc[0], W[a].sc[1] - W[b].sc[1], W[a].sc[2] - W[b].sc[2]};
                real l = sqrt(dot3(f, f));
                if (!(l > 1e-9)) { f[0] = 0; f[1] = 0; f[2] = 1; l = 1; }
                for (int k = 0; k < 3; ++k) nn[k] = f[k] / l;
                dist = 0;
            } else {
                for (int k = 0; k < 3; ++k) nn[k] /= dist;
            }
            if (deep) {
                ++g_pair_stats[5];
                if (!(m->pool_policy & 1)) continue; /* overlapping cores: no contact */
                dist = 0;
            }
            const real sep = dist - ra - rb;
            if (!(sep < off)) continue;
            PairContact *o = &out[n++];
            ++g_pair_stats[4];
            for (int k = 0; k < 3; ++k) {
                o->n[k] = nn[k];
                o->x[k] = 0.5 * ((pa[c][k] - ra * nn[k]) + (pb[c][k] + rb * nn[k]));
            }
            o->sep = sep;
            o->mu = (real)0.5 * (mu_shape[a] + mu_shape[b]);
            o->ba = ba; o->bb = bb; o->la = m->shlink[a]; o->lb = m->shlink[b];
        }
    }
    return n;
}

/* spatial inertia at O (world axes): m, h = m c, I_O (3x3) */
typedef struct { real m, h[3], I[9]; } SpI;

/* f = I * (w, v) = (I_O w + h x v, m v - h x w) */
static void spi_mul(const SpI *I, const real *mv, real *f) {
    real hv[3], hw[3], n[3];
    matvec3(I->I, mv, n);
    cross3(I->h, mv + 3, hv);
    cross3(I->h, mv, hw);
    for (int k = 0; k < 3; ++k) { f[k] = n[k] + hv[k]; f[3 + k] = I->m * mv[3 + k] - hw[k]; }
}
/* motion cross motion: (w,v) x (w',v') = (w x w', w x v' + v x w') */
static void crm(const real *a, const real *b, real *o) {
    real t1[3], t2[3], t3[3];
    cross3(a, b, t1); cross3(a, b + 3, t2); cross3(a + 3, b, t3);
    for (int k = 0; k < 3; ++k) { o[k] = t1[k]; o[3 + k] = t2[k] + t3[k]; }
}
/* motion cross force: (w,v) x* (n,f) = (w x n + v x f, w x f) */
static void crf(const real *a, const real *b, real *o) {
    real t1[3], t2[3], t3[3];
    cross3(a, b, t1); cross3(a + 3, b + 3, t2); cross3(a, b + 3, t3);
    for (int k = 0; k < 3; ++k) { o[k] = t1[k] + t2[k]; o[3 + k] = t3[k]; }
}
static inline real dot6(const real *a, const real *b) {
    real s = 0; for (int k = 0; k < 6; ++k) s += a[k] * b[k]; return s;
}

/* dense Cholesky M = L L^T in place (lower), n x n, row stride MAXV */
static void chol(real *A, int n) {
    for (int j = 0; j < n; ++j) {
        real s = A[j * MAXV + j];
        for (int k = 0; k < j; ++k) s -= A[j * MAXV + k] * A[j * MAXV + k];
        real d = sqrt(s > 0 ? s : (real)1e-30);
        A[j * MAXV + j] = d;
        for (int i = j + 1; i < n; ++i) {
            real t = A[i * MAXV + j];
            for (int k = 0; k < j; ++k) t -= A[i * MAXV + k] * A[j * MAXV + k];
            A[i * MAXV + j] = t / d;
        }
    }
}
static void chol_solve(const real *L, int n, const real *b, real *x) {
    real y[MAXV];
    for (int i = 0; i < n; ++i) {
        real t = b[i];
        for (int k = 0; k < i; ++k) t -= L[i * MAXV + k] * y[k];
        y[i] = t / L[i * MAXV + i];
    }
    for (int i = n - 1; i >= 0; --i) {
        real t = y[i];
        for (int k = i + 1; k < n; ++k) t -= L[k * MAXV + i] * x[k];
        x[i] = t / L[i * MAXV + i];
    }
}

/* ------------------------------------------------------------- one env */
static void env_substep(const OModel *m, const OParams *p, real h,
                        real *root, real *dq, const real *tau_in, const real *mu_shape,
                        real *cforce /* nb*3 or NULL */, real *sens /* nsens*6 or NULL */,
                        const real *ptgt /* nd or NULL */, const real *vtgt /* nd or NULL */)
{
    const int nb = m->nb, nd = m->nd, fb = m->fixed_base;
    const int nbase = fb ? 0 : 6, nv = nbase + nd;
    real R[MAXB][9], P[MAXB][3], S[MAXB][6], V[MAXB][6];
    SpI Ib[MAXB], Ic[MAXB];

    /* ---- forward kinematics (positions relative to the root origin) */
    {
        real q4[4] = {root[3], root[4], root[5], root[6]};
        quat_to_mat(q4, R[0]);
        P[0][0] = P[0][1] = P[0][2] = 0;
    }
    for (int i = 1; i < nb; ++i) {
        const int pa = m->parent[i];
        real Ro[9], to[3], RJ[9], a[3], tt[3];
        for (int k = 0; k < 9; ++k) Ro[k] = (real)m->jorigin[12 * i + k];
        for (int k = 0; k < 3; ++k) { to[k] = (real)m->jorigin[12 * i + 9 + k]; a[k] = (real)m->jaxis[3 * i + k]; }
        matmul3(R[pa], Ro, RJ);
        matvec3(R[pa], to, tt);
        for (int k = 0; k < 3; ++k) P[i][k] = P[pa][k] + tt[k];
        real aw[3];
        matvec3(RJ, a, aw);
        const real qj = dq[2 * m->bdof[i]];
        if (m->jkind[i] == 1) {
            real Rq[9];
            axis_angle(a, qj, Rq);
            matmul3(RJ, Rq, R[i]);
            S[i][0] = aw[0]; S[i][1] = aw[1]; S[i][2] = aw[2];
            cross3(P[i], aw, S[i] + 3);
        } else {
            memcpy(R[i], RJ, sizeof(RJ));
            for (int k = 0; k < 3; ++k) P[i][k] += aw[k] * qj;
            S[i][0] = S[i][1] = S[i][2] = 0;
            S[i][3] = aw[0]; S[i][4] = aw[1]; S[i][5] = aw[2];
        }
    }
    /* ---- spatial inertias at O */
    for (int i = 0; i < nb; ++i) {
        real c[3], cl[3], Il[9], T[9], RT[9], Iw[9];
        for (int k = 0; k < 3; ++k) cl[k] = (real)m->com[3 * i + k];
        for (int k = 0; k < 9; ++k) Il[k] = (real)m->inertia[9 * i + k];
        matvec3(R[i], cl, c);
        for (int k = 0; k < 3; ++k) c[k] += P[i][k];
        for (int a = 0; a < 3; ++a) for (int b = 0; b < 3; ++b) RT[3 * a + b] = R[i][3 * b + a];
        matmul3(R[i], Il, T);
        matmul3(T, RT, Iw);
        const real mm = (real)m->mass[i];
        const real cc = dot3(c, c);
        Ib[i].m = mm;
        for (int k = 0; k < 3; ++k) Ib[i].h[k] = mm * c[k];
        for (int a = 0; a < 3; ++a)
            for (int b = 0; b < 3; ++b)
                Ib[i].I[3 * a + b] = Iw[3 * a + b] + mm * ((a == b ? cc : 0) - c[a] * c[b]);
        Ic[i] = Ib[i];
    }
    for (int i = nb - 1; i > 0; --i) {
        const int pa = m->parent[i];
        Ic[pa].m += Ic[i].m;
        for (int k = 0; k < 3; ++k) Ic[pa].h[k] += Ic[i].h[k];
        for (int k = 0; k < 9; ++k) Ic[pa].I[k] += Ic[i].I[k];
    }

    /* ---- generalized velocity nu = (w, pdot, qd) */
    real nu[MAXV];
    if (!fb) { for (int k = 0; k < 3; ++k) { nu[k] = root[10 + k]; nu[3 + k] = root[7 + k]; } }
    for (int j = 0; j < nd; ++j) nu[nbase + j] = dq[2 * j + 1];

    /* ---- RNEA bias with gravity (A_0 = (0, -g)) */
    real A[MAXB][6], F[MAXB][6];
    for (int k = 0; k < 6; ++k) V[0][k] = 0;
    if (!fb) { for (int k = 0; k < 6; ++k) V[0][k] = nu[k]; }
    A[0][0] = A[0][1] = A[0][2] = 0;
    for (int k = 0; k < 3; ++k) A[0][3 + k] = -(real)p->gravity[k];
    for (int i = 1; i < nb; ++i) {
        const int pa = m->parent[i];
        const real qd = nu[nbase + m->bdof[i]];
        for (int k = 0; k < 6; ++k) V[i][k] = V[pa][k] + S[i][k] * qd;
        real c[6];
        crm(V[i], S[i], c);
        for (int k = 0; k < 6; ++k) A[i][k] = A[pa][k] + c[k] * qd;
    }
    for (int i = 0; i < nb; ++i) {
        real ia[6], iv[6], x[6];
        spi_mul(&Ib[i], A[i], ia);
        spi_mul(&Ib[i], V[i], iv);
        crf(V[i], iv, x);
        for (int k = 0; k < 6; ++k) F[i][k] = ia[k] + x[k];
    }
    real Fown[MAXB][6];
    memcpy(Fown, F, sizeof(F));
    for (int i = nb - 1; i > 0; --i)
        for (int k = 0; k < 6; ++k) F[m->parent[i]][k] += F[i][k];
    real bias[MAXV];
    if (!fb) for (int k = 0; k < 6; ++k) bias[k] = F[0][k];
    for (int i = 1; i < nb; ++i) bias[nbase + m->bdof[i]] = dot6(S[i], F[i]);

    /* ---- joint drives: force estimate kp (q* - q - h qd) + kd (qd* - qd); implicit
     * within the dof's effort limit, the clamped force applied explicitly when saturated */
    real dforce[MAXV];
    int dimpl[MAXV];
    if (m->dkp && m->dkd) {
        for (int j = 0; j < nd; ++j) {
            const real pt = ptgt ? ptgt[j] : 0, vt = vtgt ? vtgt[j] : 0;
            const real q = dq[2 * j], qd = dq[2 * j + 1];
            const real f = (real)m->dkp[j] * (pt - q - h * qd) + (real)m->dkd[j] * (vt - qd);
            const real ef = (real)m->effort[j];
            dimpl[j] = !(ef > 0) || fabs(f) <= ef;
            dforce[j] = dimpl[j] ? f : (f > ef ? ef : -ef);
        }
    }

    /* ---- CRBA dense mass matrix */
    real M[MAXV * MAXV];
    memset(M, 0, sizeof(M));
    if (!fb) {
        const SpI *I0 = &Ic[0];
        for (int a = 0; a < 3; ++a)
            for (int b = 0; b < 3; ++b) {
                M[a * MAXV + b] = I0->I[3 * a + b];
                M[(3 + a) * MAXV + (3 + b)] = (a == b) ? I0->m : 0;
            }
        /* upper-right block [h]x, lower-left [h]x^T */
        const real *hh = I0->h;
        real hx[9] = {0, -hh[2], hh[1], hh[2], 0, -hh[0], -hh[1], hh[0], 0};
        for (int a = 0; a < 3; ++a)
            for (int b = 0; b < 3; ++b) {
                M[a * MAXV + 3 + b] = hx[3 * a + b];
                M[(3 + b) * MAXV + a] = hx[3 * a + b];
            }
    }
    for (int i = 1; i < nb; ++i) {
        const int di = nbase + m->bdof[i];
        real Fi[6];
        spi_mul(&Ic[i], S[i], Fi);
        M[di * MAXV + di] = dot6(S[i], Fi) + (real)m->armature[m->bdof[i]];
        if (m->dkp && m->dkd && dimpl[m->bdof[i]])
            M[di * MAXV + di] += h * ((real)m->dkd[m->bdof[i]] + h * (real)m->dkp[m->bdof[i]]);
        for (int j = m->parent[i]; j > 0; j = m->parent[j]) {
            const int dj = nbase + m->bdof[j];
            const real v = dot6(S[j], Fi);
            M[di * MAXV + dj] = v; M[dj * MAXV + di] = v;
        }
        if (!fb) for (int k = 0; k < 6; ++k) { M[di * MAXV + k] = Fi[k]; M[k * MAXV + di] = Fi[k]; }
    }
    chol(M, nv);

    /* ---- free velocity */
    real rhs[MAXV], acc[MAXV], nuf[MAXV];
    for (int k = 0; k < nbase; ++k) rhs[k] = -bias[k];
    for (int j = 0; j < nd; ++j) {
        real t = tau_in[j];
        const real e = (real)m->effort[j];
        if (e > 0) t = t > e ? e : (t < -e ? -e : t);
        rhs[nbase + j] = t - bias[nbase + j];
        if (m->dkp && m->dkd) rhs[nbase + j] += dforce[j];
    }
    chol_solve(M, nv, rhs, acc);
    for (int k = 0; k < nv; ++k) nuf[k] = nu[k] + h * acc[k];
    if (!fb) {
        real wxp[3];
        cross3(nu, nu + 3, wxp);
        for (int k = 0; k < 3; ++k) nuf[3 + k] += h * wxp[k];
    }

    /* ---- joint limits: one unilateral row per dof within limit_margin of a limit,
     * J = +e (lower) / -e (upper), solved before the contacts in dof order */
    int nlim = 0, ldof[MAXV];
    real lsgn[MAXV], lsep[MAXV], LJ[MAXV * MAXV], LW[MAXV * MAXV], LD[MAXV];
    for (int j = 0; j < nd; ++j) {
        if (!(m->has_limits && m->has_limits[j] && m->upper[j] > m->lower[j])) continue;
        const real q = dq[2 * j];
        const real lo = q - (real)m->lower[j], hi = (real)m->upper[j] - q;
        if (!(lo < (real)p->limit_margin || hi < (real)p->limit_margin)) continue;
        const real sg = lo <= hi ? 1 : -1;
        real *Jr = LJ + nlim * MAXV, *Wr = LW + nlim * MAXV;
        for (int k = 0; k < nv; ++k) Jr[k] = 0;
        Jr[nbase + j] = sg;
        chol_solve(M, nv, Jr, Wr);
        LD[nlim] = sg * Wr[nbase + j];
        ldof[nlim] = j;
        lsgn[nlim] = sg;
        lsep[nlim] = lo <= hi ? lo : hi;
        ++nlim;
    }

    /* ---- contacts vs the ground plane z = 0 and the terrain mesh (deepest of the two) */
    int nact = 0;
    int ck[MAXC];
    real cs[MAXC], cmu[MAXC], cn[MAXC][3];
    const int ncap = m->nc > 0 ? m->nc : 1;
    real J[3 * ncap * MAXV], W[3 * ncap * MAXV];
    real Dr[3 * MAXC];
    int hsel[64][4], hn[64];
    if (m->shkind) {
        for (int sh = 0; sh < m->ns; ++sh) {
            hn[sh] = 0; /* a hull's ground slots: the plane only (no terrain-mesh contact) */
            if (m->shkind[sh] == 4 && p->has_ground)
                hn[sh] = hull_ground_select(m, sh, R[m->shbody[sh]], P[m->shbody[sh]], root[2], (real)p->contact_offset,
                                            hsel[sh]);
        }
    }
    if (p->has_ground || p->has_terrain) {
        for (int c = 0; c < m->nc; ++c) {
            const int b = m->cbody[c];
            real xl[3], x[3];
            for (int k = 0; k < 3; ++k) xl[k] = (real)m->cpoint[3 * c + k];
            if (m->cdyn && m->cdyn[c] >= 0) { /* a hull's ground slot: the selected vertex, if any */
                const int sh = m->cshape[c], k = m->cdyn[c];
                if (k >= hn[sh]) continue;
                for (int a = 0; a < 3; ++a) xl[a] = (real)m->hverts[4 * hsel[sh][k] + a];
            }
            matvec3(R[b], xl, x);
            for (int k = 0; k < 3; ++k) x[k] += P[b][k];
            const real r = (real)m->cradius[c];
            real dist = p->has_ground ? root[2] + x[2] - r : 1e300;
            real nrm[3] = {0, 0, 1}, smu = (real)p->ground_friction;
            if (p->has_terrain && !(m->cdyn && m->cdyn[c] >= 0)) {
                const real cw[3] = {root[0] + x[0], root[1] + x[1], root[2] + x[2]};
                real st, nt[3];
                if (terrain_query(p, cw, r, r + (real)p->contact_offset, &st, nt) && st < dist) {
                    dist = st;
                    nrm[0] = nt[0]; nrm[1] = nt[1]; nrm[2] = nt[2];
                    smu = (real)p->terrain_friction;
                }
            }
            if (!(dist < (real)p->contact_offset)) continue;
            real dir[3][3];
            for (int k = 0; k < 3; ++k) dir[0][k] = nrm[k];
            tangents(nrm, dir[1], dir[2]);
            real xc[3] = {x[0] - r * nrm[0], x[1] - r * nrm[1], x[2] - r * nrm[2]};
            real Jp[3][MAXV];
            for (int a = 0; a < 3; ++a) for (int k = 0; k < nv; ++k) Jp[a][k] = 0;
            if (!fb) {
                /* d(w x xc)/dw = -[xc]x */
                Jp[0][0] = 0;      Jp[0][1] = xc[2];  Jp[0][2] = -xc[1];
                Jp[1][0] = -xc[2]; Jp[1][1] = 0;      Jp[1][2] = xc[0];
                Jp[2][0] = xc[1];  Jp[2][1] = -xc[0]; Jp[2][2] = 0;
                Jp[0][3] = 1; Jp[1][4] = 1; Jp[2][5] = 1;
            }
            for (int i = b; i > 0; i = m->parent[i]) {
                real t[3];
                cross3(S[i], xc, t);
                const int di = nbase + m->bdof[i];
                for (int a = 0; a < 3; ++a) Jp[a][di] = S[i][3 + a] + t[a];
            }
            for (int rr = 0; rr < 3; ++rr) {
                real *Jr = J + (3 * nact + rr) * MAXV;
                real *Wr = W + (3 * nact + rr) * MAXV;
                for (int k = 0; k < nv; ++k) Jr[k] = dir[rr][0] * Jp[0][k] + dir[rr][1] * Jp[1][k] + dir[rr][2] * Jp[2][k];
                chol_solve(M, nv, Jr, Wr);
                real d = 0;
                for (int k = 0; k < nv; ++k) d += Jr[k] * Wr[k];
                Dr[3 * nact + rr] = d;
            }
            ck[nact] = c;
            cs[nact] = dist - (real)p->rest_offset;
            cmu[nact] = (real)0.5 * (mu_shape[m->cshape[c]] + smu);
            for (int k = 0; k < 3; ++k) cn[nact][k] = nrm[k];
            ++nact;
        }
    }

    /* ---- self-contacts: rows J = n.(v_A(x) - v_B(x)) over both bodies' paths (the common
     * ancestors' columns cancel), solved after the ground contacts in pool order */
    PairContact pc[MAXPOOL];
    int npc = 0;
    real PJ[3 * MAXPOOL * MAXV], PW[3 * MAXPOOL * MAXV], PD[3 * MAXPOOL];
    const real min_resp = (m->pool_policy & 2) ? (real)0 : (real)MIN_RESPONSE; /* (pool_policy bit 1: study) */
    if (m->self_collide && m->npair > 0 && m->npool > 0) {
        npc = self_contacts(m, p, R, P, mu_shape, pc);
        for (int a = 0; a < npc; ++a) {
            real dir[3][3];
            for (int k = 0; k < 3; ++k) dir[0][k] = pc[a].n[k];
            tangents(pc[a].n, dir[1], dir[2]);
            for (int rr = 0; rr < 3; ++rr) {
                real *Jr = PJ + (3 * a + rr) * MAXV, *Wr = PW + (3 * a + rr) * MAXV;
                for (int k = 0; k < nv; ++k) Jr[k] = 0;
                for (int side = 0; side < 2; ++side) {
                    const real sg = side == 0 ? 1 : -1;
                    for (int i = side == 0 ? pc[a].ba : pc[a].bb; i > 0; i = m->parent[i]) {
                        real t[3];
                        cross3(S[i], pc[a].x, t);
                        const int di = nbase + m->bdof[i];
                        Jr[di] += sg * (dir[rr][0] * (S[i][3] + t[0]) + dir[rr][1] * (S[i][4] + t[1]) +
                                        dir[rr][2] * (S[i][5] + t[2]));
                    }
                }
                chol_solve(M, nv, Jr, Wr);
                real d = 0;
                for (int k = 0; k < nv; ++k) d += Jr[k] * Wr[k];
                PD[3 * a + rr] = d;
            }
        }
    }

    /* ---- sequential impulses (joint space) */
    real v[MAXV], lam[3 * MAXC], nupos[MAXV], laml[MAXV];
    memcpy(v, nuf, sizeof(real) * nv);
    for (int k = 0; k < 3 * nact; ++k) lam[k] = 0;
    for (int k = 0; k < nlim; ++k) laml[k] = 0;
    real plam[3 * MAXPOOL];
    for (int k = 0; k < 3 * npc; ++k) plam[k] = 0;
    const int iters = p->pos_iters + p->vel_iters;
    /* TGS (solver_type 1): displacement dq integrated over the position sub-steps of length hs; a row's
     * separation is advanced by J dq (linearised), its target is set for the sub-step */
    const int tgs = p->solver_type >= 1 && p->solver_type <= 3 && p->pos_iters > 0;
    /* solver_type 3 (round 5): TGS whose position sub-steps push a penetration out at -s / h (the whole step, as
     * PGS) instead of -s / hs: the sub-steps share the push-out rather than each demanding all of it */
    const real hpush = p->solver_type == 3 ? h : (p->solver_type >= 1 && p->pos_iters > 0 ? h / p->pos_iters : h);
    /* solver_type 2 (round 5): TGS whose position sub-steps integrate the joint velocities
     * clamped to the joint velocity limits (PhysX applies maxJointVelocity in every TGS sub-step integration):
     * a row's linearised separation then advances by the displacement the clamped joints actually deliver, so
     * a sub-step push-out target the limit cannot meet is not counted as met (the round-4 divergence:
     * profiles/r04_tgs_divergence.txt) */
    const int tgs_clamp = p->solver_type == 2;
    const real hs = tgs ? h / p->pos_iters : h;
    real dxs[MAXV];
    for (int k = 0; k < nv; ++k) dxs[k] = 0;
    for (int it = 0; it < iters; ++it) {
        const int pos_phase = it < p->pos_iters;
        const real hd = pos_phase ? hs : h;  /* a separated row may close its gap within hd */
        for (int a = 0; a < nlim; ++a) {
            const real s = lsep[a] + (tgs ? lsgn[a] * dxs[nbase + ldof[a]] : 0);
            const real u = lsgn[a] * v[nbase + ldof[a]];
            real target;
            if (s >= 0) target = -s / hd;
            else if (pos_phase) { target = -s / hpush; if (target > (real)p->max_depen_vel) target = (real)p->max_depen_vel; }
            else target = 0;
            real ln = laml[a] + (target - u) / LD[a];
            if (ln < 0) ln = 0;
            const real dl = ln - laml[a];
            laml[a] = ln;
            const real *Wr = LW + a * MAXV;
            for (int k = 0; k < nv; ++k) v[k] += Wr[k] * dl;
        }
        for (int a = 0; a < nact; ++a) {
            real s = cs[a];
            /* normal */
            {
                const int r = 3 * a;
                const real *Jr = J + r * MAXV, *Wr = W + r * MAXV;
                real u = 0;
                for (int k = 0; k < nv; ++k) u += Jr[k] * v[k];
                if (tgs) for (int k = 0; k < nv; ++k) s += Jr[k] * dxs[k];
                real target;
                if (s >= 0) target = -s / hd;
                else if (pos_phase) { target = -s / hpush; if (target > (real)p->max_depen_vel) target = (real)p->max_depen_vel; }
                else target = 0;
                real ln = Dr[r] > 0 ? lam[r] + (target - u) / Dr[r] : lam[r]; /* ground rows: no response cutoff; Dr == 0: a
                                                                                  * row the articulation cannot move along */
                if (ln < 0) ln = 0;
                const real dl = ln - lam[r];
                lam[r] = ln;
                for (int k = 0; k < nv; ++k) v[k] += Wr[k] * dl;
            }
            for (int t = 1; t < 3; ++t) {
                const int r = 3 * a + t;
                const real *Jr = J + r * MAXV, *Wr = W + r * MAXV;
                real u = 0;
                for (int k = 0; k < nv; ++k) u += Jr[k] * v[k];
                const real lim = cmu[a] * lam[3 * a];
                real lt = Dr[r] > 0 ? lam[r] - u / Dr[r] : lam[r];
                if (lt > lim) lt = lim;
                if (lt < -lim) lt = -lim;
                const real dl = lt - lam[r];
                lam[r] = lt;
                for (int k = 0; k < nv; ++k) v[k] += Wr[k] * dl;
            }
        }
        for (int a = 0; a < npc; ++a) {
            real s = pc[a].sep;
            for (int t = 0; t < 3; ++t) {
                const int r = 3 * a + t;
                const real *Jr = PJ + r * MAXV, *Wr = PW + r * MAXV;
                real u = 0;
                for (int k = 0; k < nv; ++k) u += Jr[k] * v[k];
                real ln;
                if (t == 0) {
                    if (tgs) for (int k = 0; k < nv; ++k) s += Jr[k] * dxs[k];
                    real target;
                    if (s >= 0) target = -s / hd;
                    else if (pos_phase) { target = -s / hpush; if (target > (real)p->max_depen_vel) target = (real)p->max_depen_vel; }
                    else target = 0;
                    ln = PD[r] > min_resp ? plam[r] + (target - u) / PD[r] : plam[r];
                    if (ln < 0) ln = 0;
                } else {
                    const real lim = pc[a].mu * plam[3 * a];
                    ln = PD[r] > min_resp ? plam[r] - u / PD[r] : plam[r];
                    if (ln > lim) ln = lim;
                    if (ln < -lim) ln = -lim;
                }
                const real dl = ln - plam[r];
                plam[r] = ln;
                for (int k = 0; k < nv; ++k) v[k] += Wr[k] * dl;
            }
        }
        if (tgs && pos_phase) {
            if (tgs_clamp)
                for (int j = 0; j < nd; ++j) {
                    const real vm = (real)m->vmax[j];
                    if (vm > 0) {
                        real *a = &v[nbase + j];
                        if (*a > vm) *a = vm;
                        if (*a < -vm) *a = -vm;
                    }
                }
            for (int k = 0; k < nv; ++k) dxs[k] += hs * v[k];
        }
        if (it == p->pos_iters - 1) {
            if (tgs) for (int k = 0; k < nv; ++k) nupos[k] = dxs[k] / h;  /* h * nupos = the sub-steps' displacement */
            else memcpy(nupos, v, sizeof(real) * nv);
        }
    }
    if (p->pos_iters == 0) memcpy(nupos, v, sizeof(real) * nv);

    /* ---- joint velocity limits */
    for (int j = 0; j < nd; ++j) {
        const real vm = (real)m->vmax[j];
        if (vm > 0) {
            real *a = &v[nbase + j], *b = &nupos[nbase + j];
            if (*a > vm) *a = vm; if (*a < -vm) *a = -vm;
            if (*b > vm) *b = vm; if (*b < -vm) *b = -vm;
        }
    }

    /* ---- integrate positions with nu_pos, keep velocities nu_new */
    if (!fb) {
        for (int k = 0; k < 3; ++k) root[k] += h * nupos[3 + k];
        const real *w = nupos;
        real x = root[3], y = root[4], z = root[5], qw = root[6];
        real dx = 0.5 * h * (qw * w[0] + w[1] * z - w[2] * y);
        real dy = 0.5 * h * (qw * w[1] + w[2] * x - w[0] * z);
        real dz = 0.5 * h * (qw * w[2] + w[0] * y - w[1] * x);
        real dw = 0.5 * h * (-(w[0] * x + w[1] * y + w[2] * z));
        x += dx; y += dy; z += dz; qw += dw;
        const real n = 1 / sqrt(x * x + y * y + z * z + qw * qw);
        root[3] = x * n; root[4] = y * n; root[5] = z * n; root[6] = qw * n;
        for (int k = 0; k < 3; ++k) { root[10 + k] = v[k]; root[7 + k] = v[3 + k]; }
    }
    for (int j = 0; j < nd; ++j) {
        dq[2 * j] += h * nupos[nbase + j];
        dq[2 * j + 1] = v[nbase + j];
    }
    if (cforce) {
        for (int k = 0; k < 3 * m->nr; ++k) cforce[k] = 0;
        for (int a = 0; a < nact; ++a) {
            const int b = m->clink[ck[a]];
            real t1[3], t2[3];
            tangents(cn[a], t1, t2);
            for (int k = 0; k < 3; ++k)
                cforce[3 * b + k] += (lam[3 * a] * cn[a][k] + lam[3 * a + 1] * t1[k] + lam[3 * a + 2] * t2[k]) / h;
        }
        for (int a = 0; a < npc; ++a) {
            real t1[3], t2[3];
            tangents(pc[a].n, t1, t2);
            for (int k = 0; k < 3; ++k) {
                const real f = (plam[3 * a] * pc[a].n[k] + plam[3 * a + 1] * t1[k] + plam[3 * a + 2] * t2[k]) / h;
                cforce[3 * pc[a].la + k] += f;
                cforce[3 * pc[a].lb + k] -= f;
            }
        }
    }
    if (sens && m->nsens > 0) {
        /* joint-reaction wrench of each sensor (leaf) body: I a + v x* I v - f_contact, with the
         * substep's accelerations (RNEA form, gravity offset in A) -> body origin, body axes */
        real ab[6] = {0, 0, 0, 0, 0, 0};
        if (!fb) {
            real wxp[3];
            cross3(nu, nu + 3, wxp);
            for (int k = 0; k < 3; ++k) { ab[k] = (v[k] - nu[k]) / h; ab[3 + k] = (v[3 + k] - nu[3 + k]) / h - wxp[k]; }
        }
        for (int si = 0; si < m->nsens; ++si) {
            const int b = m->sens_body[si];
            real a6[6], ia[6], f[6];
            for (int k = 0; k < 6; ++k) a6[k] = ab[k];
            for (int i = b; i > 0; i = m->parent[i]) {
                const int g = nbase + m->bdof[i];
                const real qdd = (v[g] - nu[g]) / h;
                for (int k = 0; k < 6; ++k) a6[k] += S[i][k] * qdd;
            }
            spi_mul(&Ib[b], a6, ia);
            for (int k = 0; k < 6; ++k) f[k] = Fown[b][k] + ia[k];
            for (int a = 0; a < nact; ++a) {
                const int c = ck[a];
                if (m->cbody[c] != b) continue;
                real xl[3], x[3], fc[3], n[3];
                for (int k = 0; k < 3; ++k) xl[k] = (real)m->cpoint[3 * c + k];
                matvec3(R[b], xl, x);
                for (int k = 0; k < 3; ++k) x[k] += P[b][k];
                real t1[3], t2[3];
                tangents(cn[a], t1, t2);
                for (int k = 0; k < 3; ++k) {
                    x[k] -= (real)m->cradius[c] * cn[a][k];
                    fc[k] = (lam[3 * a] * cn[a][k] + lam[3 * a + 1] * t1[k] + lam[3 * a + 2] * t2[k]) / h;
                }
                cross3(x, fc, n);
                for (int k = 0; k < 3; ++k) { f[k] -= n[k]; f[3 + k] -= fc[k]; }
            }
            for (int a = 0; a < npc; ++a) {
                if (pc[a].ba != b && pc[a].bb != b) continue;
                const real sg = pc[a].ba == b ? 1 : -1;
                real t1[3], t2[3], fc[3], n3[3];
                tangents(pc[a].n, t1, t2);
                for (int k = 0; k < 3; ++k)
                    fc[k] = sg * (plam[3 * a] * pc[a].n[k] + plam[3 * a + 1] * t1[k] + plam[3 * a + 2] * t2[k]) / h;
                cross3(pc[a].x, fc, n3);
                for (int k = 0; k < 3; ++k) { f[k] -= n3[k]; f[3 + k] -= fc[k]; }
            }
            real xf[3], tq[3];
            cross3(P[b], f + 3, xf);
            for (int k = 0; k < 3; ++k) tq[k] = f[k] - xf[k];
            for (int k = 0; k < 3; ++k) {
                sens[6 * si + k] = R[b][k] * f[3] + R[b][3 + k] * f[4] + R[b][6 + k] * f[5];
                sens[6 * si + 3 + k] = R[b][k] * tq[0] + R[b][3 + k] * tq[1] + R[b][6 + k] * tq[2];
            }
        }
    }
}

/*
 * One gym.simulate() for n_envs environments.
 * root  : [N][13] pos(3) quat xyzw(4) v_origin(3) w(3)   (internal: root ORIGIN velocity)
 * dof   : [N][nd][2] (q, qd)
 * tau   : [N][nd]
 * mu    : [N][ns]     per-env shape friction
 * cf    : [N][nr][3]  net contact force per reported link (written when collect_contacts), may be NULL
 * sens  : [N][nsens][6] force-sensor readings of the last substep, may be NULL
 */
int oracle_simulate_targets(const OModel *m, const OParams *p, int n_envs, real *root, real *dof,
                            const real *tau, const real *mu, real *cf, real *sens, int num_threads,
                            const real *ptgt, const real *vtgt);

int oracle_simulate(const OModel *m, const OParams *p, int n_envs, real *root, real *dof,
                    const real *tau, const real *mu, real *cf, real *sens, int num_threads)
{
    return oracle_simulate_targets(m, p, n_envs, root, dof, tau, mu, cf, sens, num_threads, NULL, NULL);
}

/* oracle_simulate with joint-drive targets ptgt / vtgt [N][nd] (NULL = 0) */
int oracle_simulate_targets(const OModel *m, const OParams *p, int n_envs, real *root, real *dof,
                            const real *tau, const real *mu, real *cf, real *sens, int num_threads,
                            const real *ptgt, const real *vtgt)
{
    if (m->nb > MAXB || m->nd + 6 > MAXV || m->nc > MAXC || m->nr < m->nb || m->ns > 64 || m->npool > MAXPOOL) return -1;
    const real h = (real)(p->dt / (p->substeps > 0 ? p->substeps : 1));
#ifdef _OPENMP
    if (num_threads > 0) omp_set_num_threads(num_threads);
#pragma omp parallel for schedule(static)
#endif
    for (int e = 0; e < n_envs; ++e) {
        for (int s = 0; s < p->substeps; ++s) {
            const int last = (s == p->substeps - 1);
            env_substep(m, p, h, root + 13 * e, dof + 2 * m->nd * e, tau + m->nd * e, mu + m->ns * e,
                        (cf && p->collect_contacts && last) ? cf + 3 * m->nr * e : NULL,
                        (sens && last) ? sens + 6 * m->nsens * e : NULL,
                        ptgt ? ptgt + m->nd * e : NULL, vtgt ? vtgt + m->nd * e : NULL);
        }
    }
    (void)num_threads;
    return 0;
}

int oracle_real_size(void) { return (int)sizeof(real); }

/* the terrain contact query alone (test hook): out[n][5] = (found, separation, normal xyz) */
int oracle_terrain_query(const OParams *p, int n, const real *centres, const real *radii, real *out) {
    if (!p->has_terrain) return -1;
    for (int t = 0; t < n; ++t) {
        real sep = 0, nn[3] = {0, 0, 0};
        const int f = terrain_query(p, centres + 3 * t, radii[t], radii[t] + (real)p->contact_offset, &sep, nn);
        out[5 * t] = f; out[5 * t + 1] = sep; out[5 * t + 2] = nn[0]; out[5 * t + 3] = nn[1]; out[5 * t + 4] = nn[2];
    }
    return 0;
}

/* test hook: the self-contacts of each env's current state, out[n][npool][10] =
 * (x xyz, n xyz, separation, friction, body a, body b); returns per-env counts in cnt[n] */
int oracle_self_contacts(const OModel *m, const OParams *p, int n_envs, const real *root, const real *dof,
                         const real *mu, real *out, int32_t *cnt) {
    if (m->npool > MAXPOOL || m->ns > 64) return -1;
    for (int e = 0; e < n_envs; ++e) {
        const real *rt = root + 13 * e, *dq = dof + 2 * m->nd * e;
        real R[MAXB][9], P[MAXB][3];
        real q4[4] = {rt[3], rt[4], rt[5], rt[6]};
        const real qn = 1 / sqrt(q4[0] * q4[0] + q4[1] * q4[1] + q4[2] * q4[2] + q4[3] * q4[3]);
        for (int k = 0; k < 4; ++k) q4[k] *= qn;
        quat_to_mat(q4, R[0]);
        P[0][0] = P[0][1] = P[0][2] = 0;
        for (int i = 1; i < m->nb; ++i) {
            const int pa = m->parent[i];
            real Ro[9], to[3], RJ[9], a[3], tt[3];
            for (int k = 0; k < 9; ++k) Ro[k] = (real)m->jorigin[12 * i + k];
            for (int k = 0; k < 3; ++k) { to[k] = (real)m->jorigin[12 * i + 9 + k]; a[k] = (real)m->jaxis[3 * i + k]; }
            matmul3(R[pa], Ro, RJ);
            matvec3(R[pa], to, tt);
            for (int k = 0; k < 3; ++k) P[i][k] = P[pa][k] + tt[k];
            const real qj = dq[2 * m->bdof[i]];
            if (m->jkind[i] == 1) { real Rq[9]; axis_angle(a, qj, Rq); matmul3(RJ, Rq, R[i]); }
            else { real aw[3]; matvec3(RJ, a, aw); memcpy(R[i], RJ, sizeof(RJ)); for (int k = 0; k < 3; ++k) P[i][k] += aw[k] * qj; }
        }
        PairContact pc[MAXPOOL];
        const int k = self_contacts(m, p, R, P, mu + m->ns * e, pc);
        cnt[e] = k;
        for (int a = 0; a < k; ++a) {
            real *o = out + ((size_t)e * m->npool + a) * 10;
            for (int t = 0; t < 3; ++t) { o[t] = pc[a].x[t]; o[3 + t] = pc[a].n[t]; }
            o[6] = pc[a].sep; o[7] = pc[a].mu; o[8] = pc[a].ba; o[9] = pc[a].bb;
        }
    }
    return 0;
}

/* test hook: the ground contact vertices of hull shape sh for body pose (R row-major, P, root height) */
int oracle_hull_select(const OModel *m, const OParams *p, int sh, const real *R, const real *P, real rootz, int32_t *sel) {
    if (!m->shkind || sh < 0 || sh >= m->ns || m->shkind[sh] != 4) return -1;
    int s4[4];
    const int n = hull_ground_select(m, sh, R, P, rootz, (real)p->contact_offset, s4);
    for (int k = 0; k < n; ++k) sel[k] = s4[k];
    return n;
}

/* narrowphase workload counters since the last call (g_pair_stats); reset = 1 clears them */
int oracle_pair_stats(long long *out, int reset) {
    for (int i = 0; i < 7; ++i) out[i] = g_pair_stats[i];
    if (reset)
        for (int i = 0; i < 7; ++i) g_pair_stats[i] = 0;
    return 0;
}
