// host_check.cpp -- host-logic test driver (no GPU): builds a Grid from a grid file and
// reads a sim file exactly as FluidSolver does, then prints what it parsed as JSON for
// tests/test_host.py to compare with the oracle.
//   host_check <grid> [<sim>] [-no_export] [-summary]
// -no_export: the driver option (PetscInitialize) that also skips CellCenters.csv;
// -summary: print only the sizes and the peak resident set (config-size grids).
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <string>

#include "FluidSolver.h"
#include "Grid.h"
#include "sim_file.h"

int main(int argc, char** argv) {
    bool summary = false;
    for (int k = 1; k < argc; k++)
        if (!std::strcmp(argv[k], "-summary")) {
            summary = true;
            for (int q = k; q + 1 < argc; q++) argv[q] = argv[q + 1];
            argc--;
            break;
        }
    PetscInitialize(&argc, &argv, nullptr, "host_check");
    if (argc < 2) return 2;
    Grid g{argv[1]};
    if (summary) {
        // peak resident set of this image (VmHWM: getrusage's ru_maxrss would also count what
        // a forking parent held before the exec)
        long hwm = -1;
        if (FILE* f = fopen("/proc/self/status", "r")) {
            char line[256];
            while (fgets(line, sizeof line, f))
                if (!std::strncmp(line, "VmHWM:", 6)) hwm = std::atol(line + 6);
            fclose(f);
        }
        fflush(stdout);
        printf("@@JSON{\"setup\": %s, \"N\": %d, \"nx\": %d, \"ny\": %d, \"rect\": %s, \"cells_table\": %s, "
               "\"maxrss_kb\": %ld}@@\n",
               g.setup ? "true" : "false", g.N, g.nxCells(), g.nyCells(), g.isRectangle() ? "true" : "false",
               g.cells.empty() ? "false" : "true", hwm);
        return 0;
    }
    // parse the sim file first so its messages precede the JSON line
    SimParams p;
    bool ok = false, valid = false, ghosts = false;
    std::string why;
    const bool have_sim = argc >= 3 && g.setup;
    if (have_sim) {
        ok = ns_read_sim_file(argv[2], g, p);
        valid = ok && ns_check_sim_params(p);
        ghosts = valid && ns_build_ghosts(g, why);
    }
    fflush(stdout);
    printf("@@JSON{\"setup\": %s, \"N\": %d, \"nx\": %d, \"ny\": %d, \"rect\": %s", g.setup ? "true" : "false", g.N,
           g.nxCells(), g.nyCells(), g.isRectangle() ? "true" : "false");
    printf(", \"hx\": [");
    for (size_t k = 0; k < g.hx.size(); k++) printf("%s%.17g", k ? "," : "", g.hx[k]);
    printf("], \"hy\": [");
    for (size_t k = 0; k < g.hy.size(); k++) printf("%s%.17g", k ? "," : "", g.hy[k]);
    const int nx = g.setup ? g.nxCells() : 0, ny = g.setup ? g.nyCells() : 0;
    printf("], \"id\": [");
    for (int i = 0; i < nx; i++)
        for (int j = 0; j < ny; j++) printf("%s%d", i + j ? "," : "", g.cellId(i, j));
    printf("], \"tag\": [");
    for (int i = 0; i < nx; i++)
        for (int j = 0; j < ny; j++)
            for (int k = 0; k < 4; k++) printf("%s%d", i + j + k ? "," : "", g.faceEdge(i, j, k));
    printf("], \"edges\": [");
    for (size_t k = 0; k < g.edges.size(); k++)
        printf("%s[%d,%d,%.17g,%.17g,%.17g]", k ? "," : "", g.edges[k].nx, g.edges[k].ny, g.edges[k].loc[0],
               g.edges[k].loc[1], g.edges[k].loc[2]);
    printf("], \"cells_table\": %s", (!g.cells.empty() && g.cells[0][0].id == g.cellId(0, 0)) ? "true" : "false");
    if (have_sim) {
        printf(", \"sim_ok\": %s, \"sim_valid\": %s, \"ghosts\": %s, \"dt\": %.17g, \"final_time\": %.17g, \"re\": %.17g, "
               "\"saveIter\": %d, \"bc\": [",
               ok ? "true" : "false", valid ? "true" : "false", ghosts ? "true" : "false", p.dt, p.finalTime, p.re,
               p.saveIter);
        for (size_t k = 0; k < g.edges.size(); k++) {
            printf("%s[%d,%.17g", k ? "," : "", g.edges[k].bcType, g.edges[k].bcInfo);
            if (ghosts) printf(",%.17g,%.17g", g.edges[k].ghost[0].constant[0], g.edges[k].ghost[0].constant[1]);
            printf("]");
        }
        printf("]");
    }
    printf("}@@\n");
    return 0;
}
