// FluidSolver.cpp -- host side of the drop-in: reads the simulation file, validates it
// like the reference, hands the grid to libnsgpu.so (C-ABI, include/nsgpu.h) and drives
// the time loop with the reference's stdout monitor and CSV export.
// Reference behaviour cited as /root/reference/SRC/FluidSolver.cpp:<line>.
#include "FluidSolver.h"

#include <cmath>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <iostream>
#include <sstream>
#include <string>
#include <vector>

#include "nsgpu.h"
#include "sim_file.h"

namespace {

struct Options {
    int poisson = NS_POISSON_MG;
    double rtol = 1e-8;
    int device = 0;
    bool do_export = true;
};
Options g_opt;

}  // namespace

// ------------------------------------------------------------------ options
PetscErrorCode PetscInitialize(int* argc, char*** argv, const char*, const char*) {
    if (!argc || !argv) return 0;
    std::vector<char*> keep;
    keep.push_back((*argv)[0]);
    for (int k = 1; k < *argc; k++) {
        const char* a = (*argv)[k];
        auto next = [&](void) -> const char* { return k + 1 < *argc ? (*argv)[++k] : ""; };
        if (!std::strcmp(a, "-poisson")) {
            const std::string v = next();
            g_opt.poisson = v == "rbsor" ? NS_POISSON_RBSOR : v == "jacobi" ? NS_POISSON_JACOBI : NS_POISSON_MG;
        } else if (!std::strcmp(a, "-rtol")) {
            g_opt.rtol = std::atof(next());
        } else if (!std::strcmp(a, "-device")) {
            g_opt.device = std::atoi(next());
        } else if (!std::strcmp(a, "-no_export")) {
            g_opt.do_export = false;
            ns_export_files = false;   // CellCenters.csv too (Grid.cpp)
        } else {
            keep.push_back((*argv)[k]);  // positional arguments (grid file, sim file) stay
        }
    }
    for (size_t k = 0; k < keep.size(); k++) (*argv)[k] = keep[k];
    *argc = (int)keep.size();
    return 0;
}

double minmode(double a, double b) { return a * b > 0 ? a * std::fmin(1.0, std::fabs(b / a)) : 0.0; }

// ------------------------------------------------------------------ sim file (host logic)
bool ns_read_sim_file(const char* fname, Grid& grid, SimParams& p) {
    ifstream in{fname};
    if (!in) {
        cout << "Simulation data file not found!\n";
        return false;
    }
    string key, line;
    bool bad = false;
    while (!in.eof() && !bad) {
        in >> key;
        if (in.eof()) break;
        if (key == "BC") {
            // one "type info" line per edge, in the grid's edge order (FluidSolver.cpp:639-655)
            if ((in >> ws).get() != '{') { bad = true; break; }
            size_t k = 0;
            while (in.good()) {
                if ((in >> ws).peek() == '}') {
                    if (k == grid.edges.size()) in.ignore();
                    else bad = true;
                    break;
                }
                getline(in, line);
                if (in.eof() || k == grid.edges.size()) { bad = true; break; }
                istringstream ls(line);
                ls >> grid.edges[k].bcType >> grid.edges[k].bcInfo;
                k++;
            }
        } else if (key == "dt") in >> p.dt;
        else if (key == "final_time") in >> p.finalTime;
        else if (key == "re") in >> p.re;
        else if (key == "saveIter") in >> p.saveIter;
        else bad = true;
        if (!in.good()) bad = true;  // the file must end with whitespace (FluidSolver.cpp:662)
    }
    if (bad) cout << "Invalid data file format!\n";
    return !bad;
}

bool ns_check_sim_params(const SimParams& p) {
    const char* msg = nullptr;
    if (p.dt <= 0) msg = "Time step should be positive\n";
    else if (p.dt > p.finalTime) msg = "Time step should be less than final time!\n";
    else if (p.re <= 0) msg = "Reynolds number should be positive\n";
    else if (p.saveIter <= 0) msg = "saveIter must be greater than zero!\n";
    if (msg) cout << msg;
    return msg == nullptr;
}

bool ns_build_ghosts(Grid& grid, std::string& why) {
    for (size_t k = 0; k < grid.edges.size(); k++) {
        Edge& e = grid.edges[k];
        e.ghost.clear();
        const double b = e.bcInfo;
        if (e.bcType == INLET_UNI || e.bcType == WALL) {
            // velocity ghost = -q + c ; phi ghost = phi
            Stencil sv{{-1}, {{0, 0}}, {0, 0}};
            const bool normal_x = e.nx != 0;
            // inlet: the normal component carries b; wall: the tangential one (FluidSolver.cpp:89-96)
            const bool first = (e.bcType == INLET_UNI) ? normal_x : !normal_x;
            sv.constant = first ? vector<double>{2 * b, 0} : vector<double>{0, 2 * b};
            e.ghost.push_back(sv);
            e.ghost.push_back(Stencil{{1}, {{0, 0}}, {}});
        } else if (e.bcType == NEUMANN) {
            e.ghost.push_back(Stencil{{1}, {{0, 0}}, {0, 0}});
            e.ghost.push_back(Stencil{{2.5, -2.0, 0.5}, {{0, 0}, {-e.nx, -e.ny}, {-2 * e.nx, -2 * e.ny}}, {}});
        } else {
            why = "edge " + std::to_string(k) + ": boundary type " + std::to_string(e.bcType) +
                  " has no ghost stencil in the reference (INLET_PARABOLIC / PRESSURE / unset)";
            return false;
        }
    }
    return true;
}

// ------------------------------------------------------------------ solver
struct FluidSolver::Impl {
    SimParams p;
    ns_solver* gpu = nullptr;
    int nx = 0, ny = 0;
    vector<ns_edge> edges;
};

FluidSolver::FluidSolver(char* fname, Grid* g) : grid(g) {
    impl_ = new Impl();
    Impl& m = *impl_;
    if (!ns_read_sim_file(fname, *grid, m.p) || !ns_check_sim_params(m.p)) return;
    string why;
    if (!ns_build_ghosts(*grid, why)) {
        cout << "Unsupported boundary condition: " << why << "\n";
        return;
    }
    m.nx = grid->nxCells();
    m.ny = grid->nyCells();
    for (const Edge& e : grid->edges) m.edges.push_back(ns_edge{e.nx, e.ny, e.bcType, e.bcInfo});
    ns_grid_desc gd{};
    gd.nx = m.nx;
    gd.ny = m.ny;
    gd.hx = grid->hx.data();
    gd.hy = grid->hy.data();
    gd.n_edges = (int32_t)m.edges.size();
    gd.edges = m.edges.data();
    gd.cell_id = grid->isRectangle() ? nullptr : grid->cellIds().data();
    gd.face_edge = grid->isRectangle() ? nullptr : grid->faceEdges().data();
    ns_params pr{};
    pr.dt = m.p.dt;
    pr.re = m.p.re;
    pr.poisson = g_opt.poisson;
    pr.rtol = g_opt.rtol;
    pr.device = g_opt.device;
    pr.rank = 0;
    pr.nranks = 1;
    // a libnsgpu.so of another ABI would read this build's ns_params / ns_stats with other
    // layouts or enum values: refuse it (the reference's error style: message, setup = false)
    if (ns_abi_version() != NSGPU_ABI_VERSION) {
        cout << "GPU solver setup failed: libnsgpu.so has ABI " << ns_abi_version() << ", this build expects "
             << NSGPU_ABI_VERSION << "\n";
        return;
    }
    if (ns_create(&gd, &pr, &m.gpu) != 0) {
        cout << "GPU solver setup failed: " << ns_last_error() << "\n";
        return;
    }
    cout << "Solver Setup Complete!\n";
    setup = true;
}

FluidSolver::~FluidSolver() {
    if (impl_ && impl_->gpu) ns_destroy(impl_->gpu);
    delete impl_;
}

namespace {

// (L phi) and the exported pressure P = phi - dt/(2 Re) L phi (ExportData, FluidSolver.cpp:577-581)
void write_flow_csv(int iter, Grid& g, double dt, double re, const vector<double>& u, const vector<double>& v,
                    const vector<double>& phi) {
    const int nx = g.nxCells(), ny = g.nyCells();
    const double a = dt / (2 * re);
    auto id = [&](int i, int j) { return (size_t)i * ny + j; };
    char name[64];
    std::snprintf(name, sizeof name, "FlowData_%d.csv", iter);
    ofstream fs{name};
    fs << "Point_X,Point_Y,Point_Z,U,V,Pr\n";
    const int di[4] = {-1, 1, 0, 0}, dj[4] = {0, 0, -1, 1};
    for (int i = 0; i < nx; i++)
        for (int j = 0; j < ny; j++) {
            if (!g.inDomain(i, j)) continue;   // a polygon's bounding-box cells outside the domain
            const size_t c = id(i, j);
            double lap = 0.0, dg = 0.0;
            const int32_t t[4] = {g.faceEdge(i, j, 0), g.faceEdge(i, j, 1), g.faceEdge(i, j, 2), g.faceEdge(i, j, 3)};
            for (int k = 0; k < 4; k++) {
                const int ii = i + di[k], jj = j + dj[k];
                if (g.inDomain(ii, jj)) {
                    const double w = di[k] ? 2.0 / (g.hx[i] * (g.hx[i] + g.hx[ii])) : 2.0 / (g.hy[j] * (g.hy[j] + g.hy[jj]));
                    lap += w * phi[id(ii, jj)];
                    dg -= w;
                } else if (t[k] >= 0) {
                    // LHS_phi's ghost row (AddGhostStencils, FluidSolver.cpp:147-163): w (ghost - phi_c),
                    // 0 at walls / inlets, the 2.5/-2/0.5 extrapolation at a NEUMANN face
                    const Stencil& sp = g.edges[t[k]].ghost[1];
                    double gp = 0.0;
                    for (size_t q = 0; q < sp.weights.size(); q++)
                        gp += sp.weights[q] * phi[id(i + sp.support[q][0], j + sp.support[q][1])];
                    const double w = di[k] ? 1.0 / (g.hx[i] * g.hx[i]) : 1.0 / (g.hy[j] * g.hy[j]);
                    lap += w * (gp - phi[c]);
                }
            }
            lap += dg * phi[c];
            const double xc = g.centerX(i), yc = g.centerY(j);
            fs << xc << "," << yc << "," << 0.0 << "," << u[c] << "," << v[c] << "," << phi[c] + (-a) * lap << endl;
            for (int k = 0; k < 4; k++) {
                if (t[k] < 0) continue;
                const Edge& e = g.edges[t[k]];
                const Stencil& sv = e.ghost[0];
                const double gu = sv.weights[0] * u[c] + sv.constant[0];
                const double gv = sv.weights[0] * v[c] + sv.constant[1];
                double gp = 0.0;  // phi ghost (walls / inlets: phi; Neumann: extrapolation)
                const Stencil& sp = e.ghost[1];
                for (size_t q = 0; q < sp.weights.size(); q++)
                    gp += sp.weights[q] * phi[id(i + sp.support[q][0], j + sp.support[q][1])];
                fs << xc + e.nx * g.hx[i] / 2 << "," << yc + e.ny * g.hy[j] / 2 << "," << 0.0 << "," << 0.5 * (u[c] + gu)
                   << "," << 0.5 * (v[c] + gv) << "," << 0.5 * (phi[c] + gp) - dt * lap / (2 * re) << endl;
            }
        }
}

}  // namespace

void FluidSolver::Solve() {
    if (!setup) return;
    Impl& m = *impl_;
    cout << "Initiating Solver..\n";
    const size_t n = (size_t)m.nx * m.ny;
    vector<double> u, v, phi;   // host copies for the export only (allocated on the first one)
    int iter = 1;
    do {
        ns_stats st{};
        if (ns_step(m.gpu, &st) != 0) {
            cout << "Step " << iter << " failed: " << ns_last_error() << "\n";
            break;
        }
        if ((iter - 1) % 10 == 0) printf("iter\tumin\t\tumax\t\tvmin\t\tvmax\n");
        printf("%d\t%lf\t%lf\t%lf\t%lf\n", iter, st.umin, st.umax, st.vmin, st.vmax);
        if (g_opt.do_export && m.p.saveIter > 0 && iter % m.p.saveIter == 0) {
            fflush(stdout);
            if (u.empty()) u.resize(n), v.resize(n), phi.resize(n);
            // the bounding-box planes (the export's stencil walks (i, j) neighbours)
            if (ns_get_array(m.gpu, NS_ARR_U, u.data()) == 0 && ns_get_array(m.gpu, NS_ARR_V, v.data()) == 0 &&
                ns_get_array(m.gpu, NS_ARR_PHI, phi.data()) == 0)
                write_flow_csv(iter, *grid, m.p.dt, m.p.re, u, v, phi);
        }
        iter++;
    } while (m.p.dt * iter <= m.p.finalTime);
    fflush(stdout);
    cout << "Solution Complete!\n";
}
