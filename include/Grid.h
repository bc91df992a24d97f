// Grid.h -- host-side mesh for the MI355X solver, source-compatible with the
// public interface of shivams15/navierstokessolver's Grid
// (/root/reference/SRC/Grid.h:42-69): Grid(char*), setup, N, Nx, Ny, X, Y, hx,
// hy, cells, edges, ShowEdges(), inDomain(); plus the Edge / Cell / Stencil
// types and the bcTypes enum the reference's FluidSolver reads.
//
// Differences by design (DESIGN.md "Host boundary"):
//   * the mesh is also kept in compact form, which is what FluidSolver hands to
//     libnsgpu.so: a polygon keeps a cell-id plane + 4 face tags per cell (~20 B/cell);
//     a rectangle (4 edges: every cell inside) keeps nothing per cell -- its ids
//     (i*ny + j) and face tags (the side's edge) are answered by cellId() / faceEdge();
//   * the per-cell `cells` table of the reference (~190 B/cell) is only
//     materialised up to NS_GRID_CELLS_MAX cells (default 2^22 = 2048^2, ~0.8 GB);
//     above that it stays empty and `inDomain` answers from the compact form;
//   * CellCenters.csv (Grid.cpp:221-231) is skipped when the driver was started with
//     -no_export (ns_export_files, set by PetscInitialize).
#ifndef NS_AMD_GRID_H
#define NS_AMD_GRID_H

#include <cstdint>
#include <fstream>
#include <set>
#include <vector>

using namespace std;  // the reference's headers export std names to their includers

enum bcTypes : int8_t { INLET_UNI, INLET_PARABOLIC, WALL, PRESSURE, NEUMANN };
const double TOL = 1E-8;  // geometric comparison tolerance (Grid.h:7 of the reference)

// ghost value = sum(weights * value[support]) + constant[d]
struct Stencil {
    vector<double> weights;
    vector<vector<int>> support;
    vector<double> constant;
};
typedef vector<Stencil> StencilList;

struct Edge {
    int nx, ny;                    // outward normal
    vector<double> loc{0, 0, 0};   // position, start, end
    int bcType{-1};
    double bcInfo{1.0};
    StencilList ghost;             // [0] velocity, [1] phi
};
typedef vector<Edge> EdgeList;

struct Cell {
    int id{-1};
    double x, y;                       // centre
    vector<double> X{0, 0};            // west / east face x
    vector<double> Y{0, 0};            // south / north face y
    vector<int> edges{-1, -1, -1, -1}; // boundary edge on the W, E, S, N face, or -1
};
typedef vector<vector<Cell>> CellList;

class Grid {
public:
    int N = 0;                     // cells inside the domain
    vector<vector<double>> Nx;     // x segments {start, end, cells, ratio}
    vector<vector<double>> Ny;
    vector<double> X, Y;           // face coordinates
    vector<double> hx, hy;         // spacings
    CellList cells;                // reference-style table (see header note)
    EdgeList edges;
    bool setup = false;

    explicit Grid(char* fname);
    void ShowEdges(bool BC = false);
    bool inDomain(int i, int j);

    // ---- compact form used by FluidSolver / libnsgpu.so ----
    int nxCells() const { return (int)hx.size(); }
    int nyCells() const { return (int)hy.size(); }
    // polygon only (empty for a rectangle): i*ny + j -> id or -1; (i*ny + j)*4 + k -> edge or -1
    const vector<int32_t>& cellIds() const { return id_; }
    const vector<int32_t>& faceEdges() const { return tag_; }
    bool isRectangle() const { return rect_; }
    // any domain: compact id of cell (i, j) or -1; boundary edge on face k (W, E, S, N) or -1
    int32_t cellId(int i, int j) const {
        return rect_ ? (int32_t)((size_t)i * nyCells() + j) : id_[(size_t)i * nyCells() + j];
    }
    int32_t faceEdge(int i, int j, int k) const {
        if (!rect_) return tag_[((size_t)i * nyCells() + j) * 4 + k];
        const bool onside = k == 0 ? i == 0 : k == 1 ? i == nxCells() - 1 : k == 2 ? j == 0 : j == nyCells() - 1;
        return onside ? side_[k] : -1;
    }
    double centerX(int i) const { return 0.5 * (X[i] + X[i + 1]); }
    double centerY(int j) const { return 0.5 * (Y[j] + Y[j + 1]); }

private:
    vector<vector<double>> verts_;
    double xlo_ = 1E15, xhi_ = -1E15, ylo_ = 1E15, yhi_ = -1E15;
    double arlo_ = 1E15, arhi_ = -1E15;
    vector<int32_t> id_, tag_;
    bool rect_ = false;
    int32_t side_[4] = {-1, -1, -1, -1};   // rectangle: the edge on the W, E, S, N side
    bool readFile(ifstream& in);
    bool buildEdges();
    bool buildFaces();
    void classify();
    void report();
    void writeCentres();
};

bool equals(double a, double b);

// false: skip CellCenters.csv and FlowData_<iter>.csv (the -no_export option)
extern bool ns_export_files;

#endif
