/*
 * rt_bvh.cpp — host BVH builder for the triangle kernel.
 *
 * The reference has no acceleration structure: every ray scans all triangles
 * (clrt/ocl/rtcommon.h:39-68).  This binary BVH changes only which triangles a
 * ray tests, never how: leaves hold the reference's triangle_t (v0, e1, e2;
 * rtcommon.h:20-37) with the edges precomputed by the same float subtraction,
 * and the kernel's accept rule reproduces the linear loop's result exactly
 * (minimum t, ties to the highest original index).  Culling must therefore be
 * conservative: every triangle box is padded beyond the rounding slack of the
 * Moller-Trumbore test (see DESIGN.md "BVH contract").
 *
 * Binned SAH (32 bins over centroid bounds) with a depth budget: when the
 * remaining levels would only just fit a balanced tree under
 * RT_BVH_MAX_DEPTH, the split falls back to an object median, so inner depth
 * never exceeds RT_BVH_MAX_DEPTH - 1.  The cost area leans toward the scene's
 * lights (Builder::area); the 4-wide tree is the binary tree collapsed by SAH
 * dynamic programming (rt_build_bvh).
 */
#include <algorithm>
#include <array>
#include <functional>
#include <chrono>
#include <cmath>
#include <cstdlib>
#include <cstring>
#include <string>
#include <vector>

#include "rt_internal.h"
#include "rt_quant.h"

namespace {

struct Box {
    float lo[3], hi[3];
    void reset()
    {
        for (int k = 0; k < 3; ++k) {
            lo[k] = INFINITY;
            hi[k] = -INFINITY;
        }
    }
    void grow(const Box &b)
    {
        for (int k = 0; k < 3; ++k) {
            lo[k] = std::min(lo[k], b.lo[k]);
            hi[k] = std::max(hi[k], b.hi[k]);
        }
    }
    void grow(const float *p)
    {
        for (int k = 0; k < 3; ++k) {
            lo[k] = std::min(lo[k], p[k]);
            hi[k] = std::max(hi[k], p[k]);
        }
    }
};

struct TmpNode {
    Box box;
    int left = -1, right = -1; /* TmpNode indices, or -1 for a leaf */
    uint32_t first = 0, count = 0;
};

constexpr int kMaxBins = 64;

/* SAH parameters: bins per axis and the cost of one node step relative to one triangle
   test (measured on the dragon frame: 16 / 64 bins -4 / -2.5 %, node cost 0.7 / 1.5 / 1.7
   ±0.5 / -1 / -4 % against 32 and 1.0). */
int sah_bins() { return 32; }
float sah_trav() { return 1.0f; }

struct Builder {
    const float *verts;
    const int32_t *idx;
    /* The cost area of a box (SAH): the surface area — the chance that a ray of uniformly
       distributed directions meeting the parent meets it — blended with the area the box shows
       the scene's lights.  Three quarters of the dragon frame's traversal steps are shadow rays
       from mesh hits (one per light, toward it: profiles/r06s), and 4x the area projected along
       a direction is the surface-area equivalent for rays of that direction; the direction is
       taken from the centre of the box being split, averaged over the lights.  Culling only:
       any tree gives the same hits. */
    std::vector<float> lights; /* light centres, 3 per light */
    float light_w = 0.0f;      /* weight of the lights' projected area (0: surface area alone) */
    float cxy = 2.0f, cyz = 2.0f, czx = 2.0f;
    void set_weights(const Box &nb)
    {
        if (lights.empty() || light_w <= 0.0f) return;
        float m[3] = {0.0f, 0.0f, 0.0f};
        const size_t nl = lights.size() / 3;
        for (size_t l = 0; l < nl; ++l) {
            float d[3], l2 = 0.0f;
            for (int k = 0; k < 3; ++k) {
                d[k] = lights[3 * l + k] - 0.5f * (nb.lo[k] + nb.hi[k]);
                l2 += d[k] * d[k];
            }
            const float len = std::sqrt(l2);
            for (int k = 0; k < 3; ++k) m[k] += len > 0.0f ? std::fabs(d[k] / len) : 0.57735027f;
        }
        const float u = 2.0f * (1.0f - light_w), v = 4.0f * light_w / (float)nl;
        cyz = u + v * m[0];
        czx = u + v * m[1];
        cxy = u + v * m[2];
    }
    float area(const Box &bx) const
    {
        const float dx = bx.hi[0] - bx.lo[0], dy = bx.hi[1] - bx.lo[1], dz = bx.hi[2] - bx.lo[2];
        if (!(dx >= 0.0f) || !(dy >= 0.0f) || !(dz >= 0.0f)) return 0.0f;
        return cxy * dx * dy + cyz * dy * dz + czx * dz * dx;
    }
    std::vector<Box> tbox;     /* padded triangle boxes */
    std::vector<float> cent;   /* centroids, 3 per triangle */
    std::vector<uint32_t> perm;
    std::vector<TmpNode> nodes;
    uint32_t max_depth_seen = 0;

    static int ceil_log2(uint32_t v)
    {
        int l = 0;
        while ((1u << l) < v && l < 31) ++l;
        return l;
    }

    /* Levels a balanced (median) tree over n triangles needs below this node. */
    static int balanced_levels(uint32_t n)
    {
        uint32_t leaves = (n + RT_LEAF_MAX - 1) / RT_LEAF_MAX;
        return ceil_log2(leaves);
    }

    Box bounds(uint32_t first, uint32_t count) const
    {
        Box b;
        b.reset();
        for (uint32_t i = first; i < first + count; ++i) b.grow(tbox[perm[i]]);
        return b;
    }

    /* Splits [first, first+count) and returns the number in the left part, or
       0 to make a leaf. */
    uint32_t split(uint32_t first, uint32_t count, const Box &nb, uint32_t depth)
    {
        if (count <= 1) return 0;
        set_weights(nb);
        Box cb;
        cb.reset();
        for (uint32_t i = first; i < first + count; ++i) cb.grow(&cent[3 * perm[i]]);
        int axis = 0;
        float ext[3];
        for (int k = 0; k < 3; ++k) ext[k] = cb.hi[k] - cb.lo[k];
        if (ext[1] > ext[axis]) axis = 1;
        if (ext[2] > ext[axis]) axis = 2;

        const bool must_median =
            (int)depth + balanced_levels(count) >= RT_BVH_MAX_DEPTH - 1 || ext[axis] <= 0.0f;
        if (!must_median) {
            const int B = sah_bins();
            float best_cost = INFINITY;
            int best_axis = -1, best_bin = -1;
            for (int k = 0; k < 3; ++k) {
                if (!(ext[k] > 0.0f)) continue;
                Box bb[kMaxBins];
                uint32_t bn[kMaxBins];
                for (int b = 0; b < B; ++b) {
                    bb[b].reset();
                    bn[b] = 0;
                }
                const float scale = (float)B / ext[k];
                for (uint32_t i = first; i < first + count; ++i) {
                    const uint32_t t = perm[i];
                    int b = (int)((cent[3 * t + k] - cb.lo[k]) * scale);
                    b = std::min(std::max(b, 0), B - 1);
                    bb[b].grow(tbox[t]);
                    bn[b]++;
                }
                float left_area[kMaxBins];
                uint32_t left_n[kMaxBins];
                Box acc;
                acc.reset();
                uint32_t n = 0;
                for (int b = 0; b < B - 1; ++b) {
                    acc.grow(bb[b]);
                    n += bn[b];
                    left_area[b] = area(acc);
                    left_n[b] = n;
                }
                acc.reset();
                n = 0;
                for (int b = B - 1; b > 0; --b) {
                    acc.grow(bb[b]);
                    n += bn[b];
                    const uint32_t ln = left_n[b - 1];
                    if (ln == 0 || n == 0) continue;
                    const float cost = left_area[b - 1] * (float)ln + area(acc) * (float)n;
                    if (cost < best_cost) {
                        best_cost = cost;
                        best_axis = k;
                        best_bin = b;
                    }
                }
            }
            const float parent_area = area(nb);
            /* SAH: traversal cost sah_trav(), triangle cost 1 (relative to the parent) */
            const float leaf_cost = (float)count;
            const float split_cost = sah_trav() + (parent_area > 0.0f ? best_cost / parent_area : INFINITY);
            if (count <= RT_LEAF_MAX && !(split_cost < leaf_cost)) return 0;
            if (best_axis >= 0) {
                const float scale = (float)B / ext[best_axis];
                uint32_t *lo = perm.data() + first;
                uint32_t *hi = lo + count;
                uint32_t *mid = std::partition(lo, hi, [&](uint32_t t) {
                    int b = (int)((cent[3 * t + best_axis] - cb.lo[best_axis]) * scale);
                    b = std::min(std::max(b, 0), B - 1);
                    return b < best_bin;
                });
                const uint32_t nl = (uint32_t)(mid - lo);
                if (nl > 0 && nl < count) return nl;
            }
        }
        if (count <= RT_LEAF_MAX) return 0;
        /* object median along the widest centroid axis (ties broken by index) */
        const uint32_t half = count / 2;
        uint32_t *lo = perm.data() + first;
        std::nth_element(lo, lo + half, lo + count, [&](uint32_t a, uint32_t b) {
            const float ca = cent[3 * a + axis], cb2 = cent[3 * b + axis];
            return ca < cb2 || (ca == cb2 && a < b);
        });
        return half;
    }

    /* Recursive build; returns the TmpNode index. */
    int build(uint32_t first, uint32_t count, uint32_t depth)
    {
        const int id = (int)nodes.size();
        nodes.emplace_back();
        nodes[id].box = bounds(first, count);
        nodes[id].first = first;
        nodes[id].count = count;
        if (depth > max_depth_seen) max_depth_seen = depth;
        const uint32_t nl = split(first, count, nodes[id].box, depth);
        if (nl == 0) return id; /* leaf */
        const int l = build(first, nl, depth + 1);
        const int r = build(first + nl, count - nl, depth + 1);
        nodes[id].left = l;
        nodes[id].right = r;
        return id;
    }
};

int32_t leaf_code(uint32_t first, uint32_t count) { return ~(int32_t)((first << 3) | (count - 1)); }

} // namespace

bool rt_validate_mesh(const float *verts, uint32_t n_verts, const int32_t *idx, uint32_t n_tris, std::string &err)
{
    if (!verts || !idx || n_tris == 0 || n_verts == 0) {
        err = "empty mesh";
        return false;
    }
    if (n_tris >= (1u << 28)) {
        err = "too many triangles (leaf encoding holds 2^28)";
        return false;
    }
    for (uint64_t i = 0; i < 3ull * n_verts; ++i) {
        if (!std::isfinite(verts[i]) || std::fabs(verts[i]) > 1e15f) {
            err = "non-finite or out-of-range vertex coordinate";
            return false;
        }
    }
    for (uint64_t i = 0; i < 3ull * n_tris; ++i) {
        if (idx[i] < 0 || (uint32_t)idx[i] >= n_verts) {
            err = "vertex index out of range";
            return false;
        }
    }
    return true;
}

/* True when no ray of the kernel can ever accept this triangle.  Moller-Trumbore
   (geometryFuncs.h:167, rt_kernels.hip mt_test) rejects |det| < 1e-4 with
   det = dot(cross(d, e2), e1) evaluated in float.  Exactly, |det| <= |d| |e2 x e1|, and
   every query direction is unit length (camera rays, light samples, Lambert bounces:
   |d| <= 1.001 covers their rounding).  The float evaluation adds at most
   7u ||e1||_1 ||e2||_1 (u = 2^-24: two rounded products and a difference per cross
   component, then a 3-term dot); 16u is used.  The edges are the float records the
   kernel reads (e = v - v0 rounded as get_triangle does), the bound is evaluated in
   double.  Such a triangle is never hit, never occludes and never wins a tie, so
   leaving it out of the tree changes no result bit. */
static bool never_hit(const float *a, const float *p1, const float *p2)
{
    const float e1[3] = {p1[0] - a[0], p1[1] - a[1], p1[2] - a[2]};
    const float e2[3] = {p2[0] - a[0], p2[1] - a[1], p2[2] - a[2]};
    const double cx = (double)e2[1] * e1[2] - (double)e2[2] * e1[1];
    const double cy = (double)e2[2] * e1[0] - (double)e2[0] * e1[2];
    const double cz = (double)e2[0] * e1[1] - (double)e2[1] * e1[0];
    const double cr = std::sqrt(cx * cx + cy * cy + cz * cz);
    const double n1 = std::fabs((double)e1[0]) + std::fabs((double)e1[1]) + std::fabs((double)e1[2]);
    const double n2 = std::fabs((double)e2[0]) + std::fabs((double)e2[1]) + std::fabs((double)e2[2]);
    const double u = 1.0 / 16777216.0;
    const double bound = 1.001 * (cr + 16.0 * u * n1 * n2);
    return bound < 0.999 * (double)1e-4f;
}

bool rt_build_bvh(const float *verts, uint32_t n_verts, const int32_t *idx, uint32_t n_tris, RtBvh &out,
                  std::string &err)
{
    const auto t0 = std::chrono::steady_clock::now();
    if (!rt_validate_mesh(verts, n_verts, idx, n_tris, err)) return false;

    Builder b;
    b.lights = out.light_centres;
    b.light_w = out.light_cost_weight;
    b.verts = verts;
    b.idx = idx;
    b.tbox.resize(n_tris);
    b.cent.resize(3ull * n_tris);
    b.perm.resize(n_tris);
    for (uint32_t t = 0; t < n_tris; ++t) {
        Box bx;
        bx.reset();
        float maxabs = 0.0f;
        for (int k = 0; k < 3; ++k) {
            const float *p = verts + 3ull * (uint32_t)idx[3ull * t + k];
            bx.grow(p);
            for (int c = 0; c < 3; ++c) maxabs = std::max(maxabs, std::fabs(p[c]));
        }
        float ext = 0.0f;
        for (int c = 0; c < 3; ++c) ext = std::max(ext, bx.hi[c] - bx.lo[c]);
        /* culling pad: beyond the Moller-Trumbore rounding slack */
        const float pad = ext * (1.0f / 512.0f) + 1e-6f * (1.0f + maxabs);
        for (int c = 0; c < 3; ++c) {
            b.cent[3ull * t + c] = 0.5f * (bx.lo[c] + bx.hi[c]);
            bx.lo[c] -= pad;
            bx.hi[c] += pad;
        }
        b.tbox[t] = bx;
    }
    /* The tree holds the triangles a ray can hit (never_hit above), slots [0, n_hit); the
       rest follow in slots [n_hit, n_tris) for the linear traversal.  At least one
       triangle stays in the tree, so it is never empty. */
    uint32_t n_hit = 0;
    if (out.cull_unhittable) {
        std::vector<uint8_t> hit(n_tris);
        for (uint32_t t = 0; t < n_tris; ++t) {
            const float *a = verts + 3ull * (uint32_t)idx[3ull * t];
            const float *p1 = verts + 3ull * (uint32_t)idx[3ull * t + 1];
            const float *p2 = verts + 3ull * (uint32_t)idx[3ull * t + 2];
            hit[t] = !never_hit(a, p1, p2);
            n_hit += hit[t];
        }
        if (n_hit == 0) hit[0] = 1, n_hit = 1;
        for (uint32_t t = 0, k = 0, r = n_hit; t < n_tris; ++t) b.perm[hit[t] ? k++ : r++] = t;
    } else {
        n_hit = n_tris;
        for (uint32_t t = 0; t < n_tris; ++t) b.perm[t] = t;
    }
    out.n_hit = n_hit;
    b.nodes.reserve(2ull * n_hit / RT_LEAF_MAX + 16);
    const int root = b.build(0, n_hit, 1);

    /* Flatten: inner nodes in DFS preorder, each storing both children's boxes. */
    std::vector<int> order; /* TmpNode index per output inner node */
    std::vector<int> out_index(b.nodes.size(), -1);
    uint32_t n_leaves = 0;
    if (b.nodes[root].left < 0) {
        /* a single leaf: give it an inner root whose two children are that leaf */
        out.n_nodes = 1;
        out.nodes.assign(16, 0.0f);
        const Box &bx = b.nodes[root].box;
        float *n = out.nodes.data();
        n[0] = bx.lo[0]; n[1] = bx.hi[0]; n[2] = bx.lo[1]; n[3] = bx.hi[1];
        n[4] = bx.lo[0]; n[5] = bx.hi[0]; n[6] = bx.lo[1]; n[7] = bx.hi[1];
        n[8] = bx.lo[2]; n[9] = bx.hi[2]; n[10] = bx.lo[2]; n[11] = bx.hi[2];
        const int32_t code = leaf_code(0, n_hit);
        std::memcpy(&n[12], &code, 4);
        std::memcpy(&n[13], &code, 4);
        n_leaves = 1;
        out.depth = 1;
    } else {
        std::vector<int> stack;
        stack.push_back(root);
        while (!stack.empty()) {
            const int id = stack.back();
            stack.pop_back();
            out_index[id] = (int)order.size();
            order.push_back(id);
            const TmpNode &nd = b.nodes[id];
            /* push right first so the left child follows its parent */
            if (b.nodes[nd.right].left >= 0) stack.push_back(nd.right);
            if (b.nodes[nd.left].left >= 0) stack.push_back(nd.left);
        }
        out.n_nodes = (uint32_t)order.size();
        out.nodes.assign(16ull * out.n_nodes, 0.0f);
        for (uint32_t i = 0; i < out.n_nodes; ++i) {
            const TmpNode &nd = b.nodes[order[i]];
            const TmpNode &l = b.nodes[nd.left];
            const TmpNode &r = b.nodes[nd.right];
            float *n = out.nodes.data() + 16ull * i;
            n[0] = l.box.lo[0]; n[1] = l.box.hi[0]; n[2] = l.box.lo[1]; n[3] = l.box.hi[1];
            n[4] = r.box.lo[0]; n[5] = r.box.hi[0]; n[6] = r.box.lo[1]; n[7] = r.box.hi[1];
            n[8] = l.box.lo[2]; n[9] = l.box.hi[2]; n[10] = r.box.lo[2]; n[11] = r.box.hi[2];
            int32_t c0, c1;
            if (l.left >= 0) c0 = out_index[nd.left];
            else { c0 = leaf_code(l.first, l.count); ++n_leaves; }
            if (r.left >= 0) c1 = out_index[nd.right];
            else { c1 = leaf_code(r.first, r.count); ++n_leaves; }
            std::memcpy(&n[12], &c0, 4);
            std::memcpy(&n[13], &c1, 4);
        }
        /* inner depth = depth of the deepest inner node (root = 1) */
        out.depth = 0;
        std::vector<std::pair<int, uint32_t>> st;
        st.push_back({root, 1u});
        while (!st.empty()) {
            auto [id, d] = st.back();
            st.pop_back();
            const TmpNode &nd = b.nodes[id];
            if (nd.left < 0) continue;
            out.depth = std::max(out.depth, d);
            st.push_back({nd.left, d + 1});
            st.push_back({nd.right, d + 1});
        }
    }
    out.n_leaves = n_leaves;

    /* 4-wide tree: the binary tree collapsed by SAH dynamic programming over its subtrees
       (each binary node either a wide node's child — a leaf of its <= RT_LEAF_MAX triangles, or
       a wide node of its own — or dissolved into its parent's child list), costs in traversal
       steps: one per wide-node visit, one per triangle of a visited leaf (k_tris: one record per
       step), each weighted by the box's cost area (Builder::area).  Against the greedy collapse
       (expand the largest-area inner child until 4): dragon 216,474 -> 175,755 wide nodes, area
       cost -1.1 %, node visits -1.1 %, triangle tests +1.2 %, wave-steps -0.3 %, frame 85.63 ->
       85.31 ms (profiles/r06q). */
    std::vector<uint8_t> inner4(b.nodes.size(), 0); /* binary node kept as a wide node */
    std::vector<std::array<float, 5>> dcost;        /* [n][j]: n's triangles as <= j children */
    std::vector<std::array<int8_t, 5>> dsplit;      /* left share of the best j-split (0: n itself) */
    std::vector<uint8_t> as_leaf;
    {
        const size_t nn = b.nodes.size();
        dcost.assign(nn, {});
        dsplit.assign(nn, {});
        as_leaf.assign(nn, 0);
        /* children are created after their parent (build() is preorder): a reverse sweep is post-order */
        for (size_t i = nn; i-- > 0;) {
            const TmpNode &nd = b.nodes[i];
            b.set_weights(nd.box);
            const float area = b.area(nd.box);
            const float leaf_c = nd.count <= RT_LEAF_MAX ? area * (float)nd.count : INFINITY;
            if (nd.left < 0) {
                for (int j = 1; j <= 4; ++j) {
                    dcost[i][j] = leaf_c;
                    dsplit[i][j] = 0;
                }
                as_leaf[i] = 1;
                continue;
            }
            const int l = nd.left, r = nd.right;
            float best_int = INFINITY;
            for (int a = 1; a <= 3; ++a) best_int = std::min(best_int, dcost[l][a] + dcost[r][4 - a]);
            const float inner_c = area * 1.0f + best_int;
            const float self_c = std::min(leaf_c, inner_c);
            as_leaf[i] = leaf_c <= inner_c;
            dcost[i][1] = self_c;
            dsplit[i][1] = 0;
            for (int j = 2; j <= 4; ++j) {
                float best = self_c;
                int8_t arg = 0;
                for (int a = 1; a < j; ++a) {
                    const float c = dcost[l][a] + dcost[r][j - a];
                    if (c < best) {
                        best = c;
                        arg = (int8_t)a;
                    }
                }
                dcost[i][j] = best;
                dsplit[i][j] = arg;
            }
        }
    }
    {
        std::vector<int> n4_src;      /* TmpNode behind each 4-wide node */
        std::vector<int> kids_of;     /* 4 TmpNode children per 4-wide node (-1 = empty) */
        /* n's triangles as at most j children (dsplit), appended to k */
        std::function<void(int, int, int *, int &)> expand = [&](int id, int j, int *k, int &n) {
            const int a = dsplit[id][j];
            if (a == 0) {
                k[n++] = id;
                return;
            }
            expand(b.nodes[id].left, a, k, n);
            expand(b.nodes[id].right, j - a, k, n);
        };
        auto gather = [&](int id, int *kids) {
            int k[4] = {-1, -1, -1, -1};
            int n = 0;
            if (b.nodes[id].left < 0) { /* a leaf root */
                k[n++] = id;
            } else {
                const int l = b.nodes[id].left, r = b.nodes[id].right;
                int best_a = 1;
                float best = INFINITY;
                for (int a = 1; a <= 3; ++a) {
                    const float c = dcost[l][a] + dcost[r][4 - a];
                    if (c < best) {
                        best = c;
                        best_a = a;
                    }
                }
                expand(l, best_a, k, n);
                expand(r, 4 - best_a, k, n);
            }
            for (int i = 0; i < 4; ++i) {
                kids[i] = k[i];
                if (k[i] >= 0) inner4[k[i]] = !as_leaf[k[i]];
            }
        };
        /* BFS-free DFS preorder numbering */
        std::vector<int> st{root};
        inner4[root] = b.nodes[root].left >= 0;
        while (!st.empty()) {
            const int id = st.back();
            st.pop_back();
            const int me = (int)n4_src.size();
            n4_src.push_back(id);
            kids_of.resize(4 * n4_src.size());
            gather(id, &kids_of[4 * me]);
            for (int i = 3; i >= 0; --i) {
                const int c = kids_of[4 * me + i];
                if (c >= 0 && inner4[c]) st.push_back(c);
            }
        }
        std::vector<int> idx4(b.nodes.size(), -1);
        for (size_t i = 0; i < n4_src.size(); ++i) idx4[n4_src[i]] = (int)i;
        out.n_nodes4 = (uint32_t)n4_src.size();
        out.nodes4.assign(32ull * out.n_nodes4, 0.0f);
        for (uint32_t i = 0; i < out.n_nodes4; ++i) {
            float *n = out.nodes4.data() + 32ull * i;
            for (int k = 0; k < 4; ++k) {
                const int c = kids_of[4 * i + k];
                int32_t code = RT_EMPTY_CHILD;
                if (c >= 0) {
                    const TmpNode &cn = b.nodes[c];
                    n[0 + k] = cn.box.lo[0];
                    n[4 + k] = cn.box.hi[0];
                    n[8 + k] = cn.box.lo[1];
                    n[12 + k] = cn.box.hi[1];
                    n[16 + k] = cn.box.lo[2];
                    n[20 + k] = cn.box.hi[2];
                    code = inner4[c] ? idx4[c] : leaf_code(cn.first, cn.count);
                } else { /* unused slot: a zero box that is never entered (masked by the code) */
                    n[0 + k] = n[4 + k] = n[8 + k] = n[12 + k] = n[16 + k] = n[20 + k] = 0.0f;
                }
                std::memcpy(&n[24 + k], &code, 4);
            }
        }
        /* depth and worst-case stack: at a node the nearest hit child is taken
           next and up to (children - 1) are pushed; entries of all ancestors can
           be live at once. */
        out.depth4 = 0;
        out.stack4 = 0;
        std::vector<std::pair<uint32_t, std::pair<uint32_t, uint32_t>>> s4; /* node, depth, stack */
        s4.push_back({0u, {1u, 0u}});
        while (!s4.empty()) {
            auto [ni, dd] = s4.back();
            s4.pop_back();
            const uint32_t d = dd.first;
            uint32_t nk = 0;
            for (int k = 0; k < 4; ++k) nk += kids_of[4 * ni + k] >= 0;
            const uint32_t stk = dd.second + (nk > 0 ? nk - 1 : 0);
            out.depth4 = std::max(out.depth4, d);
            out.stack4 = std::max(out.stack4, stk);
            for (int k = 0; k < 4; ++k) {
                const int c = kids_of[4 * ni + k];
                if (c >= 0 && inner4[c]) s4.push_back({(uint32_t)idx4[c], {d + 1, stk}});
            }
        }
    }

    /* Renumber the 4-wide tree breadth-first with each node's inner children
       consecutive, and re-lay the triangles so each node's leaf children cover
       consecutive slots in child order (rt_quant.h); every leaf keeps its triangles
       contiguous, so the binary tree's leaf codes are remapped, not rebuilt. */
    {
        const uint32_t n4 = out.n_nodes4;
        std::vector<int32_t> new_id(n4, -1), order4;
        order4.reserve(n4);
        new_id[0] = 0;
        order4.push_back(0);
        for (size_t h = 0; h < order4.size(); ++h) {
            const float *n = out.nodes4.data() + 32ull * order4[h];
            for (int k = 0; k < 4; ++k) {
                int32_t c;
                std::memcpy(&c, &n[24 + k], 4);
                if (c != RT_EMPTY_CHILD && c >= 0) {
                    new_id[c] = (int32_t)order4.size();
                    order4.push_back(c);
                }
            }
        }
        std::vector<uint32_t> new_first(n_tris, 0u), new_perm(n_tris, 0u);
        uint32_t cursor = 0;
        for (size_t h = 0; h < order4.size(); ++h) {
            const float *n = out.nodes4.data() + 32ull * order4[h];
            for (int k = 0; k < 4; ++k) {
                int32_t c;
                std::memcpy(&c, &n[24 + k], 4);
                if (c == RT_EMPTY_CHILD || c >= 0) continue;
                const uint32_t first = (uint32_t)(~c) >> 3, count = ((uint32_t)(~c) & 7u) + 1u;
                for (uint32_t q = 0; q < count; ++q) {
                    new_first[first + q] = cursor + q; /* every slot: a merged leaf's binary leaves start inside it */
                    new_perm[cursor + q] = b.perm[first + q];
                }
                cursor += count;
            }
        }
        auto remap = [&](float *slot) {
            int32_t c;
            std::memcpy(&c, slot, 4);
            if (c == RT_EMPTY_CHILD) return;
            if (c >= 0) return;
            const uint32_t enc = (uint32_t)(~c);
            c = leaf_code(new_first[enc >> 3], (enc & 7u) + 1u);
            std::memcpy(slot, &c, 4);
        };
        std::vector<float> nodes4(out.nodes4.size());
        for (uint32_t i = 0; i < n4; ++i) {
            float *dst = nodes4.data() + 32ull * new_id[i];
            std::memcpy(dst, out.nodes4.data() + 32ull * i, 32 * sizeof(float));
            for (int k = 0; k < 4; ++k) {
                int32_t c;
                std::memcpy(&c, &dst[24 + k], 4);
                if (c != RT_EMPTY_CHILD && c >= 0) {
                    c = new_id[c];
                    std::memcpy(&dst[24 + k], &c, 4);
                } else {
                    remap(&dst[24 + k]);
                }
            }
        }
        out.nodes4.swap(nodes4);
        for (uint32_t i = 0; i < out.n_nodes; ++i) {
            remap(&out.nodes[16ull * i + 12]);
            remap(&out.nodes[16ull * i + 13]);
        }
        for (uint32_t q = cursor; q < n_tris; ++q) new_perm[q] = b.perm[q]; /* the culled tail */
        b.perm.swap(new_perm);
    }

    /* Compressed copy of the 4-wide tree (48 B per node, rt_quant.h); dropped (the
       traversal falls back to full-precision nodes) if a node cannot be encoded. */
    out.nodes4q.assign((uint64_t)RT_QNODE_DWORDS * out.n_nodes4, 0u);
    for (uint32_t i = 0; i < out.n_nodes4; ++i)
        if (!rt_quantize_node4(out.nodes4.data() + 32ull * i, out.nodes4q.data() + (uint64_t)RT_QNODE_DWORDS * i)) {
            out.nodes4q.clear();
            break;
        }

    /* Triangles in leaf order: (v0, orig), (e1 = v1 - v0), (e2 = v2 - v0). */
    out.tris.assign(12ull * n_tris, 0.0f);
    for (uint32_t s = 0; s < n_tris; ++s) {
        const uint32_t t = b.perm[s];
        const float *a = verts + 3ull * (uint32_t)idx[3ull * t];
        const float *p1 = verts + 3ull * (uint32_t)idx[3ull * t + 1];
        const float *p2 = verts + 3ull * (uint32_t)idx[3ull * t + 2];
        float *o = out.tris.data() + 12ull * s;
        o[0] = a[0];
        o[1] = a[1];
        o[2] = a[2];
        const int32_t orig = (int32_t)t;
        std::memcpy(&o[3], &orig, 4);
        o[4] = p1[0] - a[0];
        o[5] = p1[1] - a[1];
        o[6] = p1[2] - a[2];
        o[8] = p2[0] - a[0];
        o[9] = p2[1] - a[1];
        o[10] = p2[2] - a[2];
    }
    /* Normal boxes of the compressed nodes (rt_quant.h, determinant cull), bottom-up: the
       4-wide nodes are numbered breadth-first, so children follow their parents. */
    if (!out.nodes4q.empty() && out.det_cull) {
        struct NB {
            double lo[3], hi[3], err;
        };
        std::vector<NB> nb(out.n_nodes4);
        for (uint32_t i = out.n_nodes4; i-- > 0;) {
            NB b = {{INFINITY, INFINITY, INFINITY}, {-INFINITY, -INFINITY, -INFINITY}, 0.0};
            const float *f = out.nodes4.data() + 32ull * i;
            for (int k = 0; k < 4; ++k) {
                int32_t c;
                std::memcpy(&c, &f[24 + k], 4);
                if (c == RT_EMPTY_CHILD) continue;
                if (c >= 0) {
                    const NB &cb = nb[(uint32_t)c];
                    for (int a = 0; a < 3; ++a) {
                        b.lo[a] = std::min(b.lo[a], cb.lo[a]);
                        b.hi[a] = std::max(b.hi[a], cb.hi[a]);
                    }
                    b.err = std::max(b.err, cb.err);
                    continue;
                }
                const int32_t enc = ~c, first = enc >> 3, cnt = (enc & 7) + 1;
                for (int32_t j = 0; j < cnt; ++j) {
                    const float *o = out.tris.data() + 12ull * (uint32_t)(first + j);
                    const double e1[3] = {o[4], o[5], o[6]}, e2[3] = {o[8], o[9], o[10]};
                    /* N = e2 x e1 (rtcommon.h:389's normal): det = d . N */
                    const double n[3] = {e2[1] * e1[2] - e2[2] * e1[1], e2[2] * e1[0] - e2[0] * e1[2],
                                         e2[0] * e1[1] - e2[1] * e1[0]};
                    for (int a = 0; a < 3; ++a) {
                        b.lo[a] = std::min(b.lo[a], n[a]);
                        b.hi[a] = std::max(b.hi[a], n[a]);
                    }
                    const double l1 = std::fabs(e1[0]) + std::fabs(e1[1]) + std::fabs(e1[2]);
                    const double l2 = std::fabs(e2[0]) + std::fabs(e2[1]) + std::fabs(e2[2]);
                    b.err = std::max(b.err, l1 * l2);
                }
            }
            nb[i] = b;
            rt_qnode_set_nbox(out.nodes4q.data() + (uint64_t)RT_QNODE_DWORDS * i, b.lo, b.hi, b.err);
        }
    }
    out.build_seconds = std::chrono::duration<double>(std::chrono::steady_clock::now() - t0).count();
    if (out.depth >= RT_BVH_MAX_DEPTH) {
        err = "BVH deeper than the traversal stack";
        return false;
    }
    return true;
}
