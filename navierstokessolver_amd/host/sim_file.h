// sim_file.h -- simulation-file reader and the checks FluidSolver applies before setup
// (host logic; no GPU).  Format and messages follow the reference
// (/root/reference/SRC/FluidSolver.cpp:16-47, 626-669).
#pragma once
#include <string>

#include "Grid.h"

struct SimParams {
    double dt = 0.0;          // the reference leaves dt uninitialised when absent; 0 fails the check
    double finalTime = 0.0;
    double re = 0.0;
    int saveIter = 50;        // FluidSolver.h:27 default
};

// reads BC { type info (one line per grid edge) }, dt, final_time, re, saveIter into
// p and grid.edges[k].bcType / bcInfo; prints the reference's message and returns false on error
bool ns_read_sim_file(const char* fname, Grid& grid, SimParams& p);

// SolverInitialize's parameter checks; returns false (message printed) if invalid
bool ns_check_sim_params(const SimParams& p);

// ghost stencils per edge (ConstructGhostStencils, FluidSolver.cpp:84-103); returns false
// and a message for boundary types the reference cannot evaluate (INLET_PARABOLIC,
// PRESSURE, unset)
bool ns_build_ghosts(Grid& grid, std::string& why);
