// ns_main.cpp -- command-line driver: `ns_main <grid file> <sim file> [options]`.
// Same behaviour as the reference's MAIN_Solver.cpp (which also links unchanged
// against this library: see the `ref_main_link` target and INTEGRATION.md).
#include <iostream>

#include "FluidSolver.h"
#include "Grid.h"

int main(int argc, char* argv[]) {
    PetscInitialize(&argc, &argv, nullptr, "MI355X incompressible-flow solver");
    if (argc < 3) {
        std::cout << "Grid data file or simulation data file not provided!\n";
        return 0;
    }
    Grid grid{argv[1]};
    if (!grid.setup) {
        std::cout << "Grid setup failed!\n";
        return 0;
    }
    FluidSolver solver{argv[2], &grid};
    if (solver.setup) solver.Solve();
    return 0;
}
