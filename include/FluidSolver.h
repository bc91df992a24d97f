// FluidSolver.h -- the reference's solver class (/root/reference/SRC/FluidSolver.h:20-59),
// public interface unchanged: FluidSolver(char* simfile, Grid*), bool setup, void Solve().
// The time step runs on an MI355X through libnsgpu.so (include/nsgpu.h); private state
// is behind a pointer so the class stays brace-constructible on the stack exactly as
// MAIN_Solver.cpp does (MAIN_Solver.cpp:13-17).
//
// MAIN_Solver.cpp also calls PetscInitialize() without including PETSc itself, so this
// header keeps declaring PetscErrorCode / PetscInitialize (the reference got them via
// FluidSolver.h:3's petsc.h).  There is no PETSc here: PetscInitialize only reads this
// build's own options from argv (all optional):
//   -poisson mg|rbsor|jacobi   Poisson solver (default mg)
//   -rtol <x>                  relative residual of every solve (default 1e-8, the reference's KSP rtol)
//   -device <k>                HIP device (default 0)
//   -no_export                 skip FlowData_<iter>.csv
//   -quiet_grid                (ignored here; kept for symmetry with the grid output switches)
#ifndef NS_AMD_FLUIDSOLVER_H
#define NS_AMD_FLUIDSOLVER_H

#include "Grid.h"

typedef int PetscErrorCode;
PetscErrorCode PetscInitialize(int* argc, char*** argv, const char* file, const char* help);

class FluidSolver {
public:
    bool setup = false;
    FluidSolver(char* fname, Grid* grid);
    ~FluidSolver();
    FluidSolver(const FluidSolver&) = delete;
    FluidSolver& operator=(const FluidSolver&) = delete;
    void Solve();

private:
    struct Impl;
    Impl* impl_ = nullptr;
    Grid* grid;
};

// minmode limiter (FluidSolver.h:61 of the reference; the GPU kernels use the same rule)
double minmode(double a, double b);

#endif
