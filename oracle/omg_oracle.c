/* omg_oracle.c — TEST INFRASTRUCTURE ONLY (see omg_oracle.h).
 *
 * A CPU restatement of the reference octree-mg 3D hot path: ghost cells,
 * GS / GSRB smoothers, operators, restriction, prolongation and the FAS
 * V-cycle / FMG drivers.  Every function cites the reference routine it
 * restates (paths relative to the reference repository root).  Floating-point
 * expressions keep the association order that amdflang -O2 emits for the
 * reference (checked in its object code): left-to-right sums, SUM() intrinsics
 * as sequential accumulations starting from +0.0.  Built with
 * -ffp-contract=off so no FMA contraction can change a rounding.
 */
#include "omg_oracle.h"

#include <math.h>
#include <stdlib.h>
#include <string.h>

#define NB 6
#define NCH 8
#define LVL_LO (-20)
#define LVL_HI 20
#define NO_BOX 0

typedef struct {
    int n_ids, n_leaves, n_parents, n_ref_bnds;
    int *ids, *leaves, *parents, *ref_bnds;
} orc_lvl;

typedef struct {
    int bc_type;
    double bc_value;
    /* tabulated callback (per box face), or NULL */
    const long long *face_off;
    const int *face_type;
    const double *face_data;
} orc_bc;

struct orc_mg {
    int n_boxes, n_vars, n_ranks;
    int *lvl, *parent, *children, *neighbors, *ix, *rank;
    int lowest, highest, first_normal, box_size;
    int box_size_lvl[LVL_HI - LVL_LO + 1];
    double dr[LVL_HI - LVL_LO + 1][3];
    orc_lvl lvls[LVL_HI - LVL_LO + 1];
    double **cc;           /* per box (index id-1) */
    int op, smoother, n_substeps, n_cycle_down, n_cycle_up, max_coarse_cycles;
    int ahelm_fix, subtract_mean, phi_bc_data_stored;
    double lambda, res_abs, res_rel;
    orc_bc bc[NB][16];     /* bc(nb, iv) for iv < 16 */
    long long *face_off_copy[16];
    int *face_type_copy[16];
    double *face_data_copy[16];
};

/* Neighbour topology (reference: src/m_data_structures.f90:172-190). */
static const int neighb_rev[6] = {2, 1, 4, 3, 6, 5};
static const int neighb_dim[6] = {1, 1, 2, 2, 3, 3};
static const int neighb_low[6] = {1, 0, 1, 0, 1, 0};
static const int neighb_high_pm[6] = {-1, 1, -1, 1, -1, 1};

#define LV(mg, l) ((mg)->lvls[(l) - LVL_LO])
#define NCL(mg, l) ((mg)->box_size_lvl[(l) - LVL_LO])
#define DRL(mg, l) ((mg)->dr[(l) - LVL_LO])

/* cc(i,j,k,iv) of box id with box size nc: Fortran column-major. */
static inline double *ccp(const orc_mg *mg, int id, int nc, int i, int j, int k, int iv) {
    const long s = nc + 2;
    return mg->cc[id - 1] + (i + s * (j + s * (k + s * (long)(iv - 1))));
}
#define CC(id, nc, i, j, k, iv) (*ccp(mg, id, nc, i, j, k, iv))

static inline int box_nc(const orc_mg *mg, int id) { return NCL(mg, mg->lvl[id - 1]); }
static inline int nbr(const orc_mg *mg, int id, int nb) { return mg->neighbors[(id - 1) * 6 + nb - 1]; }
static inline int child(const orc_mg *mg, int id, int c) { return mg->children[(id - 1) * 8 + c - 1]; }

/* mg_get_child_offset (reference: src/m_data_structures.f90:456-467). */
static void child_offset(const orc_mg *mg, int id, int dix[3]) {
    if (mg->lvl[id - 1] <= mg->first_normal) {
        dix[0] = dix[1] = dix[2] = 0;
    } else {
        for (int d = 0; d < 3; d++) dix[d] = ((mg->ix[(id - 1) * 3 + d] - 1) & 1) * (mg->box_size >> 1);
    }
}

/* ------------------------------------------------------------------------ */
orc_mg *orc_create(int n_boxes, const int *lvl, const int *parent,
                   const int *children, const int *neighbors, const int *ix,
                   int lowest_lvl, int highest_lvl, int first_normal_lvl,
                   int box_size, const int *box_size_lvl, const double *dr,
                   const int *list_off, const int *lists, int n_vars,
                   const int *rank, int n_ranks) {
    orc_mg *mg = calloc(1, sizeof(*mg));
    mg->n_boxes = n_boxes;
    mg->n_vars = n_vars;
    mg->n_ranks = n_ranks > 0 ? n_ranks : 1;
    mg->lvl = malloc(sizeof(int) * n_boxes);
    mg->parent = malloc(sizeof(int) * n_boxes);
    mg->children = malloc(sizeof(int) * n_boxes * 8);
    mg->neighbors = malloc(sizeof(int) * n_boxes * 6);
    mg->ix = malloc(sizeof(int) * n_boxes * 3);
    mg->rank = malloc(sizeof(int) * n_boxes);
    memcpy(mg->lvl, lvl, sizeof(int) * n_boxes);
    memcpy(mg->parent, parent, sizeof(int) * n_boxes);
    memcpy(mg->children, children, sizeof(int) * n_boxes * 8);
    memcpy(mg->neighbors, neighbors, sizeof(int) * n_boxes * 6);
    memcpy(mg->ix, ix, sizeof(int) * n_boxes * 3);
    for (int b = 0; b < n_boxes; b++) mg->rank[b] = rank ? rank[b] : 0;
    mg->lowest = lowest_lvl;
    mg->highest = highest_lvl;
    mg->first_normal = first_normal_lvl;
    mg->box_size = box_size;
    for (int l = lowest_lvl; l <= highest_lvl; l++) {
        int li = l - lowest_lvl;
        NCL(mg, l) = box_size_lvl[li];
        for (int d = 0; d < 3; d++) DRL(mg, l)[d] = dr[3 * li + d];
        int *cnt[4] = {&LV(mg, l).n_ids, &LV(mg, l).n_leaves, &LV(mg, l).n_parents, &LV(mg, l).n_ref_bnds};
        int **arr[4] = {&LV(mg, l).ids, &LV(mg, l).leaves, &LV(mg, l).parents, &LV(mg, l).ref_bnds};
        for (int t = 0; t < 4; t++) {
            int a = list_off[4 * li + t], b = list_off[4 * li + t + 1];
            *cnt[t] = b - a;
            *arr[t] = malloc(sizeof(int) * (b - a + 1));
            memcpy(*arr[t], lists + a, sizeof(int) * (b - a));
        }
    }
    mg->cc = calloc(n_boxes, sizeof(double *));
    for (int l = lowest_lvl; l <= highest_lvl; l++) {
        long s = NCL(mg, l) + 2;
        for (int n = 0; n < LV(mg, l).n_ids; n++) {
            int id = LV(mg, l).ids[n];
            mg->cc[id - 1] = calloc((size_t)(s * s * s * n_vars), sizeof(double));
        }
    }
    /* defaults (reference: src/m_data_structures.f90:236-237, 307-327) */
    for (int nb = 0; nb < NB; nb++)
        for (int iv = 0; iv < 16; iv++) {
            mg->bc[nb][iv].bc_type = ORC_BC_DIRICHLET;
            mg->bc[nb][iv].bc_value = 0.0;
        }
    mg->op = ORC_LAPLACIAN;
    mg->smoother = ORC_GS;
    mg->n_substeps = 1;
    mg->n_cycle_down = 2;
    mg->n_cycle_up = 2;
    mg->max_coarse_cycles = 1000;
    mg->res_abs = 1e-8;
    mg->res_rel = 1e-8;
    return mg;
}

void orc_destroy(orc_mg *mg) {
    if (!mg) return;
    for (int b = 0; b < mg->n_boxes; b++) free(mg->cc[b]);
    free(mg->cc);
    for (int l = mg->lowest; l <= mg->highest; l++) {
        free(LV(mg, l).ids); free(LV(mg, l).leaves);
        free(LV(mg, l).parents); free(LV(mg, l).ref_bnds);
    }
    for (int iv = 0; iv < 16; iv++) {
        free(mg->face_off_copy[iv]); free(mg->face_type_copy[iv]); free(mg->face_data_copy[iv]);
    }
    free(mg->lvl); free(mg->parent); free(mg->children); free(mg->neighbors);
    free(mg->ix); free(mg->rank);
    free(mg);
}

void orc_set_operator(orc_mg *mg, int op, double lambda, int ahelm_fix) {
    mg->op = op;
    mg->lambda = lambda;
    mg->ahelm_fix = ahelm_fix;
}

/* mg_set_methods: GSRB => two substeps (reference: src/m_multigrid.f90:53-59). */
void orc_set_smoother(orc_mg *mg, int smoother, int n_cycle_down, int n_cycle_up,
                      int max_coarse_cycles, double res_abs, double res_rel) {
    mg->smoother = smoother;
    mg->n_substeps = (smoother == ORC_GSRB) ? 2 : 1;
    mg->n_cycle_down = n_cycle_down;
    mg->n_cycle_up = n_cycle_up;
    mg->max_coarse_cycles = max_coarse_cycles;
    mg->res_abs = res_abs;
    mg->res_rel = res_rel;
}

void orc_set_subtract_mean(orc_mg *mg, int on) { mg->subtract_mean = on; }

void orc_set_bc(orc_mg *mg, int iv, int nb, int bc_type, double bc_value) {
    mg->bc[nb - 1][iv - 1].bc_type = bc_type;
    mg->bc[nb - 1][iv - 1].bc_value = bc_value;
}

void orc_set_bc_faces(orc_mg *mg, int iv, const long long *face_off,
                      const int *face_type, const double *data, long long n_data) {
    int k = iv - 1;
    free(mg->face_off_copy[k]); free(mg->face_type_copy[k]); free(mg->face_data_copy[k]);
    mg->face_off_copy[k] = malloc(sizeof(long long) * mg->n_boxes * 6);
    mg->face_type_copy[k] = malloc(sizeof(int) * mg->n_boxes * 6);
    mg->face_data_copy[k] = malloc(sizeof(double) * (n_data > 0 ? n_data : 1));
    memcpy(mg->face_off_copy[k], face_off, sizeof(long long) * mg->n_boxes * 6);
    memcpy(mg->face_type_copy[k], face_type, sizeof(int) * mg->n_boxes * 6);
    if (n_data > 0) memcpy(mg->face_data_copy[k], data, sizeof(double) * n_data);
    for (int nb = 0; nb < NB; nb++) {
        mg->bc[nb][k].face_off = mg->face_off_copy[k];
        mg->bc[nb][k].face_type = mg->face_type_copy[k];
        mg->bc[nb][k].face_data = mg->face_data_copy[k];
    }
}

void orc_get_box(const orc_mg *mg, int id, int iv, double *out) {
    int nc = box_nc(mg, id);
    long s = nc + 2, n = s * s * s;
    memcpy(out, mg->cc[id - 1] + n * (iv - 1), sizeof(double) * n);
}

void orc_set_box(orc_mg *mg, int id, int iv, const double *in) {
    int nc = box_nc(mg, id);
    long s = nc + 2, n = s * s * s;
    memcpy(mg->cc[id - 1] + n * (iv - 1), in, sizeof(double) * n);
}

/* ------------------------------------------------------------------------ */
/* Face access.  A face array gc(a,b) (a fastest) holds, for x faces gc(j,k),
 * for y faces gc(i,k), for z faces gc(i,j) (reference:
 * src/m_ghost_cells.f90:456-497 box_gc_for_neighbor, :579-663 get/set). */
static inline double *face_cell(orc_mg *mg, int id, int nc, int nb, int layer, int a, int b, int iv) {
    /* layer: index along the face normal (0..nc+1) */
    switch (neighb_dim[nb - 1]) {
    case 1: return ccp(mg, id, nc, layer, a, b, iv);
    case 2: return ccp(mg, id, nc, a, layer, b, iv);
    default: return ccp(mg, id, nc, a, b, layer, iv);
    }
}

/* box_gc_for_neighbor (reference: src/m_ghost_cells.f90:456-497). */
static void box_gc_for_neighbor(orc_mg *mg, int id, int nb, int nc, int iv, double *gc) {
    int layer = neighb_low[nb - 1] ? 1 : nc;
    for (int b = 1; b <= nc; b++)
        for (int a = 1; a <= nc; a++) gc[(a - 1) + nc * (b - 1)] = *face_cell(mg, id, nc, nb, layer, a, b, iv);
}

/* box_get_gc / box_set_gc (reference: src/m_ghost_cells.f90:579-663). */
static void box_get_gc(orc_mg *mg, int id, int nb, int nc, int iv, double *gc) {
    int layer = neighb_low[nb - 1] ? 0 : nc + 1;
    for (int b = 1; b <= nc; b++)
        for (int a = 1; a <= nc; a++) gc[(a - 1) + nc * (b - 1)] = *face_cell(mg, id, nc, nb, layer, a, b, iv);
}

static void box_set_gc(orc_mg *mg, int id, int nb, int nc, int iv, const double *gc) {
    int layer = neighb_low[nb - 1] ? 0 : nc + 1;
    for (int b = 1; b <= nc; b++)
        for (int a = 1; a <= nc; a++) *face_cell(mg, id, nc, nb, layer, a, b, iv) = gc[(a - 1) + nc * (b - 1)];
}

/* box_gc_for_fine_neighbor (reference: src/m_ghost_cells.f90:500-577):
 * the coarse face slab tmp(0:hnc+1,0:hnc+1) next to the fine box, linearly
 * interpolated in the two tangential directions. */
static void box_gc_for_fine_neighbor(orc_mg *mg, int id, int nb, const int di[3], int nc, int iv, double *gc) {
    int hnc = nc / 2, ts = hnc + 2;
    double *tmp = malloc(sizeof(double) * ts * ts);
    int layer = neighb_low[nb - 1] ? 1 : nc;
    for (int b = 0; b <= hnc + 1; b++)
        for (int a = 0; a <= hnc + 1; a++) {
            double v;
            switch (neighb_dim[nb - 1]) {
            case 1: v = CC(id, nc, layer, di[1] + a, di[2] + b, iv); break;
            case 2: v = CC(id, nc, di[0] + a, layer, di[2] + b, iv); break;
            default: v = CC(id, nc, di[0] + a, di[1] + b, layer, iv); break;
            }
            tmp[a + ts * b] = v;
        }
#define T(a, b) tmp[(a) + ts * (b)]
    for (int j = 1; j <= hnc; j++)
        for (int i = 1; i <= hnc; i++) {
            double g1 = 0.125 * (T(i + 1, j) - T(i - 1, j));
            double g2 = 0.125 * (T(i, j + 1) - T(i, j - 1));
            gc[(2 * i - 2) + nc * (2 * j - 2)] = T(i, j) - g1 - g2;
            gc[(2 * i - 1) + nc * (2 * j - 2)] = T(i, j) + g1 - g2;
            gc[(2 * i - 2) + nc * (2 * j - 1)] = T(i, j) - g1 + g2;
            gc[(2 * i - 1) + nc * (2 * j - 1)] = T(i, j) + g1 + g2;
        }
#undef T
    free(tmp);
}

/* sides_rb (reference: src/m_ghost_cells.f90:769-861). */
static void sides_rb(orc_mg *mg, int id, int nc, int iv, int nb, const double *gc) {
    int x1 = neighb_low[nb - 1] ? 1 : nc;
    int d = neighb_low[nb - 1] ? 1 : -1;
    for (int b = 1; b <= nc; b++)
        for (int a = 1; a <= nc; a++) {
            double *g = face_cell(mg, id, nc, nb, x1 - d, a, b, iv);
            double v1 = *face_cell(mg, id, nc, nb, x1, a, b, iv);
            double v2 = *face_cell(mg, id, nc, nb, x1 + d, a, b, iv);
            *g = 0.5 * gc[(a - 1) + nc * (b - 1)] + 0.75 * v1 - 0.25 * v2;
        }
}

/* bc_to_gc (reference: src/m_ghost_cells.f90:665-766). */
static void bc_to_gc(orc_mg *mg, int id, int nc, int iv, int nb, int bc_type) {
    double c0, c1, c2;
    switch (bc_type) {
    case ORC_BC_DIRICHLET: c0 = 2; c1 = -1; c2 = 0; break;
    case ORC_BC_NEUMANN:
        c0 = DRL(mg, mg->lvl[id - 1])[neighb_dim[nb - 1] - 1] * (double)neighb_high_pm[nb - 1];
        c1 = 1; c2 = 0; break;
    case ORC_BC_CONTINUOUS: c0 = 0; c1 = 2; c2 = -1; break;
    default: abort(); /* error stop "bc_to_gc: unknown boundary condition" */
    }
    int g = neighb_low[nb - 1] ? 0 : nc + 1;
    int x1 = neighb_low[nb - 1] ? 1 : nc;
    int x2 = neighb_low[nb - 1] ? 2 : nc - 1;
    for (int b = 1; b <= nc; b++)
        for (int a = 1; a <= nc; a++) {
            double *pg = face_cell(mg, id, nc, nb, g, a, b, iv);
            *pg = c0 * *pg + c1 * *face_cell(mg, id, nc, nb, x1, a, b, iv) +
                  c2 * *face_cell(mg, id, nc, nb, x2, a, b, iv);
        }
}

/* Physical bc values of one face: the callback (tabulated) or bc_value. */
static int bc_values(orc_mg *mg, int id, int nb, int nc, int iv, double *bc) {
    const orc_bc *B = &mg->bc[nb - 1][iv - 1];
    if (B->face_off && B->face_off[(id - 1) * 6 + nb - 1] >= 0) {
        memcpy(bc, B->face_data + B->face_off[(id - 1) * 6 + nb - 1], sizeof(double) * nc * nc);
        return B->face_type[(id - 1) * 6 + nb - 1];
    }
    for (int n = 0; n < nc * nc; n++) bc[n] = B->bc_value;
    return B->bc_type;
}

/* fill_refinement_bnd (reference: src/m_ghost_cells.f90:287-328), 1 rank. */
static void fill_refinement_bnd(orc_mg *mg, int id, int nb, int nc, int iv, double *gc) {
    int p_id = mg->parent[id - 1];
    int p_nb_id = nbr(mg, p_id, nb);
    int off[3];
    child_offset(mg, id, off);
    box_gc_for_fine_neighbor(mg, p_nb_id, neighb_rev[nb - 1], off, nc, iv, gc);
    sides_rb(mg, id, nc, iv, nb, gc);
}

/* set_ghost_cells (reference: src/m_ghost_cells.f90:232-285), 1 rank. */
static void set_ghost_cells(orc_mg *mg, int id, int nc, int iv, double *gc) {
    for (int nb = 1; nb <= NB; nb++) {
        int nb_id = nbr(mg, id, nb);
        if (nb_id > NO_BOX) {
            box_gc_for_neighbor(mg, nb_id, neighb_rev[nb - 1], nc, iv, gc);
            box_set_gc(mg, id, nb, nc, iv, gc);
        } else if (nb_id == NO_BOX) {
            fill_refinement_bnd(mg, id, nb, nc, iv, gc);
        } else {
            int bc_type;
            if (mg->phi_bc_data_stored && iv == 1) {
                box_get_gc(mg, id, nb, nc, 2, gc);
                bc_type = nb_id;
            } else {
                bc_type = bc_values(mg, id, nb, nc, iv, gc);
            }
            box_set_gc(mg, id, nb, nc, iv, gc);
            bc_to_gc(mg, id, nc, iv, nb, bc_type);
        }
    }
}

/* mg_fill_ghost_cells_lvl (reference: src/m_ghost_cells.f90:131-175). */
void orc_fill_ghost_cells_lvl(orc_mg *mg, int lvl, int iv) {
    int nc = NCL(mg, lvl);
    double *gc = malloc(sizeof(double) * nc * nc);
    for (int n = 0; n < LV(mg, lvl).n_ids; n++) set_ghost_cells(mg, LV(mg, lvl).ids[n], nc, iv, gc);
    free(gc);
}

/* mg_fill_ghost_cells (reference: src/m_ghost_cells.f90:120-128). */
void orc_fill_ghost_cells(orc_mg *mg, int iv) {
    for (int l = mg->lowest; l <= mg->highest; l++) orc_fill_ghost_cells_lvl(mg, l, iv);
}

/* mg_phi_bc_store (reference: src/m_ghost_cells.f90:66-117). */
void orc_phi_bc_store(orc_mg *mg) {
    for (int l = mg->lowest; l <= mg->highest; l++) {
        int nc = NCL(mg, l);
        double *bc = malloc(sizeof(double) * nc * nc);
        for (int n = 0; n < LV(mg, l).n_ids; n++) {
            int id = LV(mg, l).ids[n];
            for (int nb = 1; nb <= NB; nb++) {
                if (nbr(mg, id, nb) < NO_BOX) {
                    int t = bc_values(mg, id, nb, nc, 1, bc);
                    mg->neighbors[(id - 1) * 6 + nb - 1] = t;
                    box_set_gc(mg, id, nb, nc, 2, bc);
                }
            }
        }
        free(bc);
    }
    mg->phi_bc_data_stored = 1;
}

/* ------------------------------------------------------------------------ */
/* Operators and smoothers. */

/* idr2 = 1/dr**2 and the sum() of three (reference: m_laplacian.f90:64-65). */
static void idr2_of(const orc_mg *mg, int lvl, double idr2[3]) {
    for (int d = 0; d < 3; d++) idr2[d] = 1 / (DRL(mg, lvl)[d] * DRL(mg, lvl)[d]);
}

/* box_gs_lpl / box_gs_helmh (reference: src/m_laplacian.f90:52-114,
 * src/m_helmholtz.f90:49-108): cell update iff (i+j+k+n) even for GSRB. */
static void box_gs_const(orc_mg *mg, int id, int nc, int cntr) {
    double idr2[3], fac;
    idr2_of(mg, mg->lvl[id - 1], idr2);
    if (mg->op == ORC_HELMHOLTZ)
        fac = 1.0 / (2 * ((idr2[0] + idr2[1]) + idr2[2]) + mg->lambda);
    else
        fac = 0.5 / ((idr2[0] + idr2[1]) + idr2[2]);
    int rb = (mg->smoother == ORC_GSRB), di = rb ? 2 : 1, i0 = 1;
    for (int k = 1; k <= nc; k++)
        for (int j = 1; j <= nc; j++) {
            if (rb) i0 = 2 - ((cntr ^ (k + j)) & 1);
            for (int i = i0; i <= nc; i += di) {
                CC(id, nc, i, j, k, 1) =
                    fac * (idr2[0] * (CC(id, nc, i + 1, j, k, 1) + CC(id, nc, i - 1, j, k, 1)) +
                           idr2[1] * (CC(id, nc, i, j + 1, k, 1) + CC(id, nc, i, j - 1, k, 1)) +
                           idr2[2] * (CC(id, nc, i, j, k + 1, 1) + CC(id, nc, i, j, k - 1, 1)) -
                           CC(id, nc, i, j, k, 2));
            }
        }
}

/* box_gs_ahelmh (reference: src/m_ahelmholtz.f90:69-162).  The reference's 3D
 * branch stores eps3 into a0(4:5) (line 145), clobbering a0(4) and leaving
 * a0(6) undefined; the result is NaN there.  This restatement implements the
 * evident intent a0(5:6) = eps3 (as the operator box_ahelmh, line 221, does).
 * Parity for this smoother is therefore unpinned against the reference. */
static void box_gs_ahelm(orc_mg *mg, int id, int nc, int cntr) {
    /* m_vlaplacian / m_vhelmholtz (src/m_vlaplacian.f90:51-131,
     * src/m_vhelmholtz.f90:61-141) are the same update with one coefficient
     * eps (var 5) for all directions; vlaplacian divides by sum(c) alone. */
    const int v = (mg->op == ORC_AHELMHOLTZ);
    const int e1 = 5, e2 = v ? 6 : 5, e3 = v ? 7 : 5;
    const double lam = (mg->op == ORC_VLAPLACIAN) ? 0.0 : mg->lambda;
    double idr2[6];
    const double *d = DRL(mg, mg->lvl[id - 1]);
    for (int q = 0; q < 3; q++) idr2[2 * q] = idr2[2 * q + 1] = 1 / (d[q] * d[q]);
    int rb = (mg->smoother == ORC_GSRB), di = rb ? 2 : 1, i0 = 1;
    for (int k = 1; k <= nc; k++)
        for (int j = 1; j <= nc; j++) {
            if (rb) i0 = 2 - ((cntr ^ (k + j)) & 1);
            for (int i = i0; i <= nc; i += di) {
                double a0[6], a[6], u[6], c[6];
                a0[0] = a0[1] = CC(id, nc, i, j, k, e1);
                a0[2] = a0[3] = CC(id, nc, i, j, k, e2);
                a0[4] = a0[5] = CC(id, nc, i, j, k, e3);
                u[0] = CC(id, nc, i - 1, j, k, 1); u[1] = CC(id, nc, i + 1, j, k, 1);
                a[0] = CC(id, nc, i - 1, j, k, e1); a[1] = CC(id, nc, i + 1, j, k, e1);
                u[2] = CC(id, nc, i, j - 1, k, 1); u[3] = CC(id, nc, i, j + 1, k, 1);
                a[2] = CC(id, nc, i, j - 1, k, e2); a[3] = CC(id, nc, i, j + 1, k, e2);
                u[4] = CC(id, nc, i, j, k - 1, 1); u[5] = CC(id, nc, i, j, k + 1, 1);
                a[4] = CC(id, nc, i, j, k - 1, e3); a[5] = CC(id, nc, i, j, k + 1, e3);
                double scu = 0.0, sc = 0.0;
                for (int q = 0; q < 6; q++) c[q] = 2 * a0[q] * a[q] / (a0[q] + a[q]) * idr2[q];
                for (int q = 0; q < 6; q++) scu += c[q] * u[q];
                for (int q = 0; q < 6; q++) sc += c[q];
                if (mg->op == ORC_VLAPLACIAN)
                    CC(id, nc, i, j, k, 1) = (scu - CC(id, nc, i, j, k, 2)) / sc;
                else
                    CC(id, nc, i, j, k, 1) = (scu - CC(id, nc, i, j, k, 2)) / (sc + lam);
            }
        }
}

void orc_box_smoother(orc_mg *mg, int id, int cntr) {
    int nc = box_nc(mg, id);
    if (mg->op == ORC_AHELMHOLTZ || mg->op == ORC_VLAPLACIAN || mg->op == ORC_VHELMHOLTZ)
        box_gs_ahelm(mg, id, nc, cntr);
    else
        box_gs_const(mg, id, nc, cntr);
}

/* box_lpl / box_helmh / box_ahelmh / box_vlpl / box_vhelmh (reference:
 * src/m_laplacian.f90:155-195, src/m_helmholtz.f90:111-154,
 * src/m_ahelmholtz.f90:165-237, src/m_vlaplacian.f90:134-189,
 * src/m_vhelmholtz.f90:144-205). */
void orc_box_op(orc_mg *mg, int id, int i_out) {
    int nc = box_nc(mg, id);
    double idr2[3];
    idr2_of(mg, mg->lvl[id - 1], idr2);
    if (mg->op == ORC_AHELMHOLTZ || mg->op == ORC_VLAPLACIAN || mg->op == ORC_VHELMHOLTZ) {
        const int v = (mg->op == ORC_AHELMHOLTZ);
        const int e1 = 5, e2 = v ? 6 : 5, e3 = v ? 7 : 5;
        double i2[6];
        for (int q = 0; q < 3; q++) i2[2 * q] = i2[2 * q + 1] = idr2[q];
        for (int k = 1; k <= nc; k++)
            for (int j = 1; j <= nc; j++)
                for (int i = 1; i <= nc; i++) {
                    double u0 = CC(id, nc, i, j, k, 1), a0[6], u[6], a[6];
                    a0[0] = a0[1] = CC(id, nc, i, j, k, e1);
                    a0[2] = a0[3] = CC(id, nc, i, j, k, e2);
                    a0[4] = a0[5] = CC(id, nc, i, j, k, e3);
                    u[0] = CC(id, nc, i - 1, j, k, 1); u[1] = CC(id, nc, i + 1, j, k, 1);
                    u[2] = CC(id, nc, i, j - 1, k, 1); u[3] = CC(id, nc, i, j + 1, k, 1);
                    u[4] = CC(id, nc, i, j, k - 1, 1); u[5] = CC(id, nc, i, j, k + 1, 1);
                    a[0] = CC(id, nc, i - 1, j, k, e1); a[1] = CC(id, nc, i + 1, j, k, e1);
                    a[2] = CC(id, nc, i, j - 1, k, e2); a[3] = CC(id, nc, i, j + 1, k, e2);
                    a[4] = CC(id, nc, i, j, k - 1, e3); a[5] = CC(id, nc, i, j, k + 1, e3);
                    double s = 0.0;
                    for (int q = 0; q < 6; q++) s += 2 * i2[q] * a0[q] * a[q] / (a0[q] + a[q]) * (u[q] - u0);
                    CC(id, nc, i, j, k, i_out) = (mg->op == ORC_VLAPLACIAN) ? s : s - mg->lambda * u0;
                }
        return;
    }
    for (int k = 1; k <= nc; k++)
        for (int j = 1; j <= nc; j++)
            for (int i = 1; i <= nc; i++) {
                double u = CC(id, nc, i, j, k, 1);
                double v = idr2[0] * (CC(id, nc, i - 1, j, k, 1) + CC(id, nc, i + 1, j, k, 1) - 2 * u) +
                           idr2[1] * (CC(id, nc, i, j - 1, k, 1) + CC(id, nc, i, j + 1, k, 1) - 2 * u) +
                           idr2[2] * (CC(id, nc, i, j, k - 1, 1) + CC(id, nc, i, j, k + 1, 1) - 2 * u);
                if (mg->op == ORC_HELMHOLTZ) v = v - mg->lambda * u;
                CC(id, nc, i, j, k, i_out) = v;
            }
}

/* mg_apply_op (reference: src/m_multigrid.f90:439-456). */
void orc_apply_op(orc_mg *mg, int i_out) {
    for (int l = mg->lowest; l <= mg->highest; l++)
        for (int n = 0; n < LV(mg, l).n_ids; n++) orc_box_op(mg, LV(mg, l).ids[n], i_out);
}

/* residual_box (reference: src/m_multigrid.f90:426-436). */
static void residual_box(orc_mg *mg, int id, int nc) {
    orc_box_op(mg, id, 4);
    for (int k = 1; k <= nc; k++)
        for (int j = 1; j <= nc; j++)
            for (int i = 1; i <= nc; i++)
                CC(id, nc, i, j, k, 4) = CC(id, nc, i, j, k, 2) - CC(id, nc, i, j, k, 4);
}

void orc_residual_lvl(orc_mg *mg, int lvl) {
    int nc = NCL(mg, lvl);
    for (int n = 0; n < LV(mg, lvl).n_ids; n++) residual_box(mg, LV(mg, lvl).ids[n], nc);
}

/* max_residual_lvl (reference: src/m_multigrid.f90:296-311). */
double orc_max_residual_lvl(orc_mg *mg, int lvl) {
    int nc = NCL(mg, lvl);
    double mx = 0.0;
    for (int n = 0; n < LV(mg, lvl).n_ids; n++) {
        int id = LV(mg, lvl).ids[n];
        residual_box(mg, id, nc);
        double r = 0.0;
        for (int k = 1; k <= nc; k++)
            for (int j = 1; j <= nc; j++)
                for (int i = 1; i <= nc; i++) {
                    double a = fabs(CC(id, nc, i, j, k, 4));
                    if (a > r) r = a;
                }
        if (r > mx) mx = r;
    }
    return mx;
}

/* ------------------------------------------------------------------------ */
/* restrict_onto (reference: src/m_restrict.f90:165-214): coarse cell =
 * 0.125 * SUM over the 2x2x2 fine cells, column-major, from +0.0. */
static void restrict_onto(orc_mg *mg, int id, int nc, int iv) {
    int hnc = nc / 2, ncp = NCL(mg, mg->lvl[id - 1]);
    for (int c = 1; c <= NCH; c++) {
        int c_id = child(mg, id, c);
        if (c_id == NO_BOX) continue;
        int dix[3];
        child_offset(mg, c_id, dix);
        for (int k = 1; k <= hnc; k++)
            for (int j = 1; j <= hnc; j++)
                for (int i = 1; i <= hnc; i++) {
                    double s = 0.0;
                    for (int kk = 2 * k - 1; kk <= 2 * k; kk++)
                        for (int jj = 2 * j - 1; jj <= 2 * j; jj++)
                            for (int ii = 2 * i - 1; ii <= 2 * i; ii++) s += CC(c_id, nc, ii, jj, kk, iv);
                    CC(id, ncp, dix[0] + i, dix[1] + j, dix[2] + k, iv) = 0.125 * s;
                }
    }
}

/* mg_restrict_lvl (reference: src/m_restrict.f90:83-114), 1 rank. */
void orc_restrict_lvl(orc_mg *mg, int iv, int lvl) {
    if (lvl <= mg->lowest) abort(); /* error stop "cannot restrict lvl <= lowest_lvl" */
    int nc = NCL(mg, lvl);
    for (int n = 0; n < LV(mg, lvl - 1).n_parents; n++) restrict_onto(mg, LV(mg, lvl - 1).parents[n], nc, iv);
}

/* mg_restrict (reference: src/m_restrict.f90:72-80). */
void orc_restrict(orc_mg *mg, int iv) {
    for (int l = mg->highest; l >= mg->lowest + 1; l--) orc_restrict_lvl(mg, iv, l);
}

/* mg_prolong_sparse (reference: src/m_prolong.f90:159-240). */
static void prolong_sparse(orc_mg *mg, int p_id, const int dix[3], int nc, int iv, double *fine) {
    int hnc = nc / 2, ncp = NCL(mg, mg->lvl[p_id - 1]);
#define F(i, j, k) fine[((i) - 1) + nc * (((j) - 1) + nc * ((k) - 1))]
    for (int k = 1; k <= hnc; k++) {
        int kc = k + dix[2];
        for (int j = 1; j <= hnc; j++) {
            int jc = j + dix[1];
            for (int i = 1; i <= hnc; i++) {
                int ic = i + dix[0];
                double f0 = 0.25 * CC(p_id, ncp, ic, jc, kc, iv);
                double flx = 0.25 * CC(p_id, ncp, ic - 1, jc, kc, iv);
                double fhx = 0.25 * CC(p_id, ncp, ic + 1, jc, kc, iv);
                double fly = 0.25 * CC(p_id, ncp, ic, jc - 1, kc, iv);
                double fhy = 0.25 * CC(p_id, ncp, ic, jc + 1, kc, iv);
                double flz = 0.25 * CC(p_id, ncp, ic, jc, kc - 1, iv);
                double fhz = 0.25 * CC(p_id, ncp, ic, jc, kc + 1, iv);
                F(2 * i - 1, 2 * j - 1, 2 * k - 1) = f0 + flx + fly + flz;
                F(2 * i, 2 * j - 1, 2 * k - 1) = f0 + fhx + fly + flz;
                F(2 * i - 1, 2 * j, 2 * k - 1) = f0 + flx + fhy + flz;
                F(2 * i, 2 * j, 2 * k - 1) = f0 + fhx + fhy + flz;
                F(2 * i - 1, 2 * j - 1, 2 * k) = f0 + flx + fly + fhz;
                F(2 * i, 2 * j - 1, 2 * k) = f0 + fhx + fly + fhz;
                F(2 * i - 1, 2 * j, 2 * k) = f0 + flx + fhy + fhz;
                F(2 * i, 2 * j, 2 * k) = f0 + fhx + fhy + fhz;
            }
        }
    }
#undef F
}

/* mg_prolong + prolong_onto (reference: src/m_prolong.f90:51-85,124-156). */
void orc_prolong(orc_mg *mg, int lvl, int iv, int iv_to, int add) {
    if (lvl == mg->highest) abort(); /* error stop "cannot prolong highest level" */
    int nc = NCL(mg, lvl + 1);
    double *tmp = malloc(sizeof(double) * nc * nc * nc);
    for (int n = 0; n < LV(mg, lvl + 1).n_ids; n++) {
        int id = LV(mg, lvl + 1).ids[n], dix[3];
        child_offset(mg, id, dix);
        prolong_sparse(mg, mg->parent[id - 1], dix, nc, iv, tmp);
        for (int k = 1; k <= nc; k++)
            for (int j = 1; j <= nc; j++)
                for (int i = 1; i <= nc; i++) {
                    double t = tmp[(i - 1) + nc * ((j - 1) + nc * (k - 1))];
                    if (add) CC(id, nc, i, j, k, iv_to) = CC(id, nc, i, j, k, iv_to) + t;
                    else CC(id, nc, i, j, k, iv_to) = t;
                }
    }
    free(tmp);
}

/* ------------------------------------------------------------------------ */
/* smooth_boxes (reference: src/m_multigrid.f90:404-424). */
void orc_smooth_boxes(orc_mg *mg, int lvl, int n_cycle) {
    for (int n = 1; n <= n_cycle * mg->n_substeps; n++) {
        for (int q = 0; q < LV(mg, lvl).n_ids; q++) orc_box_smoother(mg, LV(mg, lvl).ids[q], n);
        orc_fill_ghost_cells_lvl(mg, lvl, 1);
    }
}

/* update_coarse (reference: src/m_multigrid.f90:347-384). */
void orc_update_coarse(orc_mg *mg, int lvl) {
    int nc = NCL(mg, lvl), ncc = NCL(mg, lvl - 1);
    for (int n = 0; n < LV(mg, lvl).n_ids; n++) residual_box(mg, LV(mg, lvl).ids[n], nc);
    orc_restrict_lvl(mg, 1, lvl);
    orc_restrict_lvl(mg, 4, lvl);
    orc_fill_ghost_cells_lvl(mg, lvl - 1, 1);
    long s = ncc + 2, n3 = s * s * s;
    for (int n = 0; n < LV(mg, lvl - 1).n_parents; n++) {
        int id = LV(mg, lvl - 1).parents[n];
        orc_box_op(mg, id, 2);
        for (int k = 1; k <= ncc; k++)
            for (int j = 1; j <= ncc; j++)
                for (int i = 1; i <= ncc; i++)
                    CC(id, ncc, i, j, k, 2) = CC(id, ncc, i, j, k, 2) + CC(id, ncc, i, j, k, 4);
        memcpy(mg->cc[id - 1] + 2 * n3, mg->cc[id - 1], sizeof(double) * n3);
    }
}

/* correct_children (reference: src/m_multigrid.f90:387-402). */
void orc_correct_children(orc_mg *mg, int lvl) {
    int nc = NCL(mg, lvl);
    long s = nc + 2, n3 = s * s * s;
    for (int n = 0; n < LV(mg, lvl).n_parents; n++) {
        double *c = mg->cc[LV(mg, lvl).parents[n] - 1];
        for (long q = 0; q < n3; q++) c[3 * n3 + q] = c[q] - c[2 * n3 + q];
    }
    orc_prolong(mg, lvl, 4, 1, 1);
}

/* get_sum (reference: src/m_multigrid.f90:278-294) for the leaves of one
 * rank, in my_leaves order. */
static double get_sum_rank(orc_mg *mg, int iv, int r) {
    double s = 0.0;
    for (int l = 1; l <= mg->highest; l++) {
        int nc = NCL(mg, l);
        double w = DRL(mg, l)[0] * DRL(mg, l)[1] * DRL(mg, l)[2];
        for (int n = 0; n < LV(mg, l).n_leaves; n++) {
            int id = LV(mg, l).leaves[n];
            if (mg->rank[id - 1] != r) continue;
            double b = 0.0;
            for (int k = 1; k <= nc; k++)
                for (int j = 1; j <= nc; j++)
                    for (int i = 1; i <= nc; i++) b += CC(id, nc, i, j, k, iv);
            s = s + w * b;
        }
    }
    return s;
}

/* MPI_Allreduce(sum) of one double over n ranks is a
 * binomial tree in rank order, ((a0+a1)+(a2+a3))+a4 ...: MPICH 3.3.2 on one node
 * reduces to rank 0 along a binomial tree before the broadcast (pinned by the
 * golden runs at 1-6 and 8 ranks); for 1 rank it is the value itself. */
static double allreduce_sum(const double *v, int n) {
    double *t = malloc(sizeof(double) * n);
    memcpy(t, v, sizeof(double) * n);
    for (int w = 1; w < n; w *= 2)
        for (int r = 0; r + w < n; r += 2 * w) t[r] = t[r] + t[r + w];
    double s = t[0];
    free(t);
    return s;
}

double orc_get_sum(orc_mg *mg, int iv) {
    double *p = malloc(sizeof(double) * mg->n_ranks);
    for (int r = 0; r < mg->n_ranks; r++) p[r] = get_sum_rank(mg, iv, r);
    double s = allreduce_sum(p, mg->n_ranks);
    free(p);
    return s;
}

/* subtract_mean (reference: src/m_multigrid.f90:245-276). */
void orc_subtract_mean(orc_mg *mg, int iv, int include_ghostcells) {
    int nc = mg->box_size;
    double mean = orc_get_sum(mg, iv);
    double volume = (double)(nc * nc * nc) * (DRL(mg, 1)[0] * DRL(mg, 1)[1] * DRL(mg, 1)[2]) *
                    (double)LV(mg, 1).n_ids;
    mean = mean / volume;
    for (int l = mg->lowest; l <= mg->highest; l++) {
        int ncl = NCL(mg, l);
        for (int n = 0; n < LV(mg, l).n_ids; n++) {
            int id = LV(mg, l).ids[n];
            if (include_ghostcells) {
                for (int k = 0; k <= ncl + 1; k++)
                    for (int j = 0; j <= ncl + 1; j++)
                        for (int i = 0; i <= ncl + 1; i++) CC(id, ncl, i, j, k, iv) = CC(id, ncl, i, j, k, iv) - mean;
            } else {
                for (int k = 1; k <= ncl; k++)
                    for (int j = 1; j <= ncl; j++)
                        for (int i = 1; i <= ncl; i++) CC(id, ncl, i, j, k, iv) = CC(id, ncl, i, j, k, iv) - mean;
            }
        }
    }
}

/* mg_fas_vcycle (reference: src/m_multigrid.f90:150-243). */
void orc_fas_vcycle(orc_mg *mg, int highest_lvl, int want_max_res, double *max_res, int standalone) {
    int has_highest = highest_lvl >= mg->lowest;
    if (mg->subtract_mean && !has_highest) orc_subtract_mean(mg, 2, 0);
    int min_lvl = mg->lowest, max_lvl = has_highest ? highest_lvl : mg->highest;
    if (standalone) orc_fill_ghost_cells_lvl(mg, max_lvl, 1);
    for (int l = max_lvl; l >= min_lvl + 1; l--) {
        orc_smooth_boxes(mg, l, mg->n_cycle_down);
        orc_update_coarse(mg, l);
    }
    double init_res = orc_max_residual_lvl(mg, min_lvl), res;
    for (int i = 1; i <= mg->max_coarse_cycles; i++) {
        orc_smooth_boxes(mg, min_lvl, mg->n_cycle_up + mg->n_cycle_down);
        res = orc_max_residual_lvl(mg, min_lvl);
        if (res < mg->res_rel * init_res || res < mg->res_abs) break;
    }
    for (int l = min_lvl + 1; l <= max_lvl; l++) {
        orc_correct_children(mg, l - 1);
        orc_fill_ghost_cells_lvl(mg, l, 1);
        orc_smooth_boxes(mg, l, mg->n_cycle_up);
    }
    if (want_max_res) {
        init_res = 0.0;
        for (int l = min_lvl; l <= max_lvl; l++) {
            res = orc_max_residual_lvl(mg, l);
            init_res = (res > init_res) ? res : init_res;
        }
        *max_res = init_res;
    }
    if (mg->subtract_mean) orc_subtract_mean(mg, 1, 1);
}

/* mg_fas_fmg (reference: src/m_multigrid.f90:84-147). */
void orc_fas_fmg(orc_mg *mg, int have_guess, int want_max_res, double *max_res) {
    if (!have_guess) {
        for (int l = mg->highest; l >= mg->lowest; l--) {
            long s = NCL(mg, l) + 2, n3 = s * s * s;
            for (int n = 0; n < LV(mg, l).n_ids; n++) memset(mg->cc[LV(mg, l).ids[n] - 1], 0, sizeof(double) * n3);
        }
    }
    orc_fill_ghost_cells_lvl(mg, mg->highest, 1);
    for (int l = mg->highest; l >= mg->lowest + 1; l--) orc_update_coarse(mg, l);
    if (mg->subtract_mean) orc_subtract_mean(mg, 2, 0);
    for (int l = mg->lowest; l <= mg->highest; l++) {
        long s = NCL(mg, l) + 2, n3 = s * s * s;
        for (int n = 0; n < LV(mg, l).n_ids; n++) {
            double *c = mg->cc[LV(mg, l).ids[n] - 1];
            memcpy(c + 2 * n3, c, sizeof(double) * n3);
        }
        if (l > mg->lowest) {
            orc_correct_children(mg, l - 1);
            orc_fill_ghost_cells_lvl(mg, l, 1);
        }
        if (l == mg->highest) orc_fas_vcycle(mg, l, want_max_res, max_res, 0);
        else orc_fas_vcycle(mg, l, 0, NULL, 0);
    }
}

/* set_rhs of m_diffusion (reference: src/m_diffusion.f90:144-159):
 * rhs = f1*phi + f2*rhs on the interior of the leaves of levels 1..highest. */
void orc_set_rhs(orc_mg *mg, double f1, double f2) {
    for (int l = 1; l <= mg->highest; l++) {
        int nc = NCL(mg, l);
        for (int n = 0; n < LV(mg, l).n_leaves; n++) {
            int id = LV(mg, l).leaves[n];
            for (int k = 1; k <= nc; k++)
                for (int j = 1; j <= nc; j++)
                    for (int i = 1; i <= nc; i++)
                        CC(id, nc, i, j, k, 2) = f1 * CC(id, nc, i, j, k, 1) + f2 * CC(id, nc, i, j, k, 2);
        }
    }
}

/* diffusion_solve / _vcoeff / _acoeff (reference: src/m_diffusion.f90:19-57,
 * :63-101, :108-142).  op selects the variant (helmholtz: lambda from
 * 1/(dt*D); vhelmholtz / ahelmholtz: 1/dt, pass D = 1).  Returns 0, or
 * 1 "no convergence" (after 10 V-cycles), 2 "order should be 1 or 2". */
int orc_diffusion_solve(orc_mg *mg, int op, double dt, double coeff, int order, double max_res,
                        int *n_vcycles, double *res_out) {
    if (order != 1 && order != 2) return 2;                 /* :42-43 */
    double dtc = op == ORC_HELMHOLTZ ? dt * coeff : dt;
    mg->op = op;                                            /* :29-30, mg_set_methods */
    if (op != ORC_AHELMHOLTZ) mg->subtract_mean = 0;        /* m_helmholtz.f90:21, m_vhelmholtz.f90:28 */
    if (order == 1) {                                       /* :33-35 */
        mg->lambda = 1 / dtc;
        orc_set_rhs(mg, -1 / dtc, 0.0);
    } else {                                                /* :36-40 */
        mg->lambda = 0.0;
        orc_apply_op(mg, 2);
        mg->lambda = 2 / dtc;
        orc_set_rhs(mg, -2 / dtc, -1.0);
    }
    double res = 0.0;
    orc_fas_fmg(mg, 1, 1, &res);                            /* :47 */
    int n;
    for (n = 1; n <= 10; n++) {                             /* :50-53 */
        if (res <= max_res) break;
        orc_fas_vcycle(mg, mg->lowest - 1, 1, &res, 1);
    }
    if (n_vcycles) *n_vcycles = n - 1;
    if (res_out) *res_out = res;
    return n == 11 ? 1 : 0;                                 /* :55-58 */
}
