// Grid.cpp -- host mesh builder (API: include/Grid.h).  Behaviour follows the
// reference's Grid (/root/reference/SRC/Grid.cpp): same input format and
// messages, same face / cell construction and compact id order, so cell ids,
// boundary tags and CellCenters.csv are interchangeable.  Storage is compact.
#include "Grid.h"

#include <algorithm>
#include <cmath>
#include <cstdlib>
#include <iomanip>
#include <iostream>
#include <sstream>
#include <string>

bool equals(double a, double b) { return std::fabs(a - b) <= TOL; }

bool ns_export_files = true;

namespace {

// read "{ row ; row ; ... }" where each row fills up to `width` numbers (missing
// trailing numbers keep their default -1: Grid.cpp:260-264)
bool read_rows(ifstream& in, vector<vector<double>>& rows, size_t width, bool linewise) {
    if ((in >> ws).get() != '{') return false;
    string line;
    while (in.good()) {
        if ((in >> ws).peek() == '}') { in.ignore(); return true; }
        rows.push_back(vector<double>(width, linewise ? -1.0 : 0.0));
        if (linewise) {
            getline(in, line);
            istringstream ls(line);
            for (size_t k = 0; k < width && (ls >> rows.back()[k]); k++) {}
        } else {
            for (size_t k = 0; k < width; k++) in >> rows.back()[k];
        }
        if (in.eof()) return false;
    }
    return true;
}

// one axis of GenerateFaces (Grid.cpp:78-120): uniform (ratio -1) or geometric (ratio > 0)
bool faces_along(vector<vector<double>>& segs, vector<double>& F, vector<double>& H, double& h) {
    for (auto& s : segs) {
        if (!equals(s[0], F.back()) || (F.size() == 1 && s[2] <= 0)) return false;
        const double len = s[1] - s[0], r = s[3];
        if (r > 0) {
            if (s[2] <= 0) s[2] = std::ceil(std::log(len * (r - 1) / h + 1) / std::log(r));
            h = len * (r - 1) / (std::pow(r, s[2]) - 1);
        } else if (r == -1) {
            if (s[2] <= 0) s[2] = std::ceil(len / h);
            h = len / s[2];
        } else {
            return false;
        }
        double x = s[0];
        for (int k = 0; k < s[2]; k++) {
            x += h;
            F.push_back(x);
            H.push_back(h);
            if (r > 0) h *= r;
        }
    }
    return true;
}

}  // namespace

Grid::Grid(char* fname) {
    ifstream in{fname};
    if (readFile(in)) {
        if (buildEdges() && buildFaces()) {
            classify();
            report();
            setup = true;
        }
    }
    in.close();
    writeCentres();  // written even when setup failed (Grid.cpp:15)
}

bool Grid::readFile(ifstream& in) {
    if (!in) {
        cout << "Grid data file not found!\n";
        return false;
    }
    string key;
    bool ok = true;
    while (!in.eof()) {
        in >> key;
        if (in.eof()) break;
        if (key == "Vertices") ok = read_rows(in, verts_, 2, false);
        else if (key == "Nx") ok = read_rows(in, Nx, 4, true);
        else if (key == "Ny") ok = read_rows(in, Ny, 4, true);
        else ok = false;
        if (!ok || !in.good()) { ok = false; break; }
    }
    if (!ok) cout << "Invalid data file format!\n";
    return ok;
}

// GenerateEdges (Grid.cpp:28-72): the polygon is closed back to its first vertex;
// a clockwise walk gives outward normals as below.
bool Grid::buildEdges() {
    cout << "Generating Edges...\n";
    if (verts_.empty()) return false;
    const size_t nv = verts_.size();
    for (size_t k = 0; k < nv; k++) {
        const vector<double>& a = verts_[k];
        const vector<double>& b = verts_[(k + 1) % nv];
        Edge e;
        e.nx = e.ny = 0;
        if (b[0] == a[0]) {
            e.loc = {b[0], std::min(a[1], b[1]), std::max(a[1], b[1])};
            e.nx = b[1] > a[1] ? -1 : 1;
            if (e.nx < 0) xlo_ = std::min(xlo_, b[0]); else xhi_ = std::max(xhi_, b[0]);
        } else if (b[1] == a[1]) {
            e.loc = {b[1], std::min(a[0], b[0]), std::max(a[0], b[0])};
            e.ny = b[0] > a[0] ? 1 : -1;
            if (e.ny > 0) yhi_ = std::max(yhi_, b[1]); else ylo_ = std::min(ylo_, b[1]);
        } else {
            cout << "Edges should be parallel to the x-axis or y-axis\n";
            return false;
        }
        edges.push_back(e);
    }
    return true;
}

bool Grid::buildFaces() {
    cout << "Generating Faces...\n";
    X.assign(1, xlo_);
    Y.assign(1, ylo_);
    double h = 0.0;  // carried across segments and axes, as in the reference
    bool ok = faces_along(Nx, X, hx, h) && faces_along(Ny, Y, hy, h);
    ok = ok && equals(xhi_, X.back()) && equals(yhi_, Y.back());
    if (!ok) cout << "Invalid specification for number of cells\n";
    return ok;
}

// GenerateCells + Cleanup + Interior (Grid.cpp:131-185): ray cast along +x counts
// crossings of vertical edges; faces lying on an edge get that edge's index.
// A 4-edge polygon is a rectangle (every cell inside, ids i*ny + j, each side one edge):
// nothing is stored per cell, cellId() / faceEdge() answer from the side table.
void Grid::classify() {
    cout << "Generating Cells...\n";
    const int nx = nxCells(), ny = nyCells();
    const int ne = (int)edges.size();
    if (ne == 4) {
        rect_ = true;
        N = nx * ny;
        const int snx[4] = {-1, 1, 0, 0}, sny[4] = {0, 0, -1, 1};
        for (int k = 0; k < ne; k++)
            for (int f = 0; f < 4; f++)
                if (edges[k].nx == snx[f] && edges[k].ny == sny[f]) side_[f] = k;
        // the aspect-ratio range of the cells: min / max of (xe - xw) / (yn - ys) (monotone
        // in each factor, so the extremes pair the extreme widths and heights)
        double dxlo = 1E300, dxhi = -1E300, dylo = 1E300, dyhi = -1E300;
        for (int i = 0; i < nx; i++) dxlo = std::min(dxlo, X[i + 1] - X[i]), dxhi = std::max(dxhi, X[i + 1] - X[i]);
        for (int j = 0; j < ny; j++) dylo = std::min(dylo, Y[j + 1] - Y[j]), dyhi = std::max(dyhi, Y[j + 1] - Y[j]);
        arlo_ = dxlo / dyhi;
        arhi_ = dxhi / dylo;
    } else {
        id_.assign((size_t)nx * ny, -1);
        tag_.assign((size_t)nx * ny * 4, -1);
        int n = 0;
        for (int i = 0; i < nx; i++) {
            const double xw = X[i], xe = X[i + 1], xc = 0.5 * (xw + xe);
            for (int j = 0; j < ny; j++) {
                const double ys = Y[j], yn = Y[j + 1], yc = 0.5 * (ys + yn);
                int32_t* t = &tag_[((size_t)i * ny + j) * 4];
                int crossings = 0;
                for (int k = 0; k < ne; k++) {
                    const Edge& e = edges[k];
                    if (e.nx != 0) {
                        if (!(yc > e.loc[1] && yc < e.loc[2])) continue;
                        if (e.loc[0] > xc) crossings++;
                        if (e.nx == -1 && equals(xw, e.loc[0])) t[0] = k;
                        if (e.nx == 1 && equals(xe, e.loc[0])) t[1] = k;
                    } else {
                        if (!(xc > e.loc[1] && xc < e.loc[2])) continue;
                        if (e.ny == -1 && equals(ys, e.loc[0])) t[2] = k;
                        if (e.ny == 1 && equals(yn, e.loc[0])) t[3] = k;
                    }
                }
                if (crossings % 2) {
                    id_[(size_t)i * ny + j] = n++;
                    const double ar = (xe - xw) / (yn - ys);
                    arlo_ = std::min(arlo_, ar);
                    arhi_ = std::max(arhi_, ar);
                }
            }
        }
        N = n;
    }
    const char* cap = getenv("NS_GRID_CELLS_MAX");
    const long long cellsMax = cap ? atoll(cap) : (1LL << 22);
    if ((long long)nx * ny > cellsMax) return;  // compact form only
    cells.assign(nx, vector<Cell>(ny));
    for (int i = 0; i < nx; i++)
        for (int j = 0; j < ny; j++) {
            Cell& c = cells[i][j];
            c.X = {X[i], X[i + 1]};
            c.Y = {Y[j], Y[j + 1]};
            c.x = 0.5 * (X[i] + X[i + 1]);
            c.y = 0.5 * (Y[j] + Y[j + 1]);
            c.id = cellId(i, j);
            c.edges = {faceEdge(i, j, 0), faceEdge(i, j, 1), faceEdge(i, j, 2), faceEdge(i, j, 3)};
        }
}

void Grid::report() {
    cout << setprecision(2);
    ShowEdges();
    cout << endl;
    cout << "X:\t" << xlo_ << "\t" << xhi_ << endl;
    cout << "Y:\t" << ylo_ << "\t" << yhi_ << endl;
    cout << "AR:\t" << arlo_ << "\t" << arhi_ << endl;
    cout << "hx:\t" << *min_element(hx.begin(), hx.end()) << "\t" << *max_element(hx.begin(), hx.end()) << endl;
    cout << "hy:\t" << *min_element(hy.begin(), hy.end()) << "\t" << *max_element(hy.begin(), hy.end()) << endl
         << endl;
}

void Grid::ShowEdges(bool BC) {
    cout << endl;
    for (size_t k = 0; k < edges.size(); k++) {
        const Edge& e = edges[k];
        cout << "Edge\t" << k << ":\tn\t" << e.nx << "\t" << e.ny << "\t";
        if (e.nx != 0) cout << "x\t" << e.loc[0] << "\ty\t" << e.loc[1] << "\t" << e.loc[2] << endl;
        else cout << "y\t" << e.loc[0] << "\tx\t" << e.loc[1] << "\t" << e.loc[2] << endl;
        if (BC) cout << "BC\t" << e.bcType << "\t" << e.bcInfo << endl;
    }
}

bool Grid::inDomain(int i, int j) {
    if (i < 0 || j < 0 || i >= nxCells() || j >= nyCells()) return false;
    return cellId(i, j) >= 0;
}

void Grid::writeCentres() {
    if (!ns_export_files) return;   // -no_export
    ofstream out{"CellCenters.csv"};
    const int nx = nxCells(), ny = nyCells();
    if (!setup) return;   // (the reference writes an empty file when setup failed)
    for (int i = 0; i < nx; i++)
        for (int j = 0; j < ny; j++)
            if (cellId(i, j) != -1) out << centerX(i) << "," << centerY(j) << "\n";
}
