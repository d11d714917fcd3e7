// Uses include/nuSIprop.hpp exactly like the reference's test.cpp uses its
// header (test.cpp:6-33), plus the mutable members, the copy constructor and
// the range-checked getters.  Built by tests/test_facade.py.
#include <cstdio>

#include "nuSIprop.hpp"

static void dump(const char* tag, nuSIprop::calculate_flux& ev)
{
    for (int i = 0; i < ev.get_N_bins_E(); ++i)
        printf("%s %.17e %.17e %.17e %.17e\n", tag, ev.get_energy(i), ev.get_flux_fla(0, i), ev.get_flux_fla(1, i),
               ev.get_flux_fla(2, i));
}

int main()
{
    nuSIprop::calculate_flux evolver(6e5, 0.01, 0.1, 2.5, 6, true, true, true, 100, 9, 14, 5, 2, false);
    evolver.evolve();
    dump("A", evolver);
    nuSIprop::calculate_flux other(evolver);   // deep copy keeps the fluxes
    other.g = 0.05;                            // public member, re-read by evolve()
    other.mphi = 2e6;
    other.evolve();
    dump("B", other);
    dump("C", evolver);                        // the original is untouched
    printf("R %.17e\n", evolver.get_flux(0, -1) + evolver.get_flux_fla(3, 0) + evolver.get_energy(1000));
    // BASELINE config 2a (DSNB, the resonance inside lE 4 -> 9, N_E = 300) with no option: the reference's arithmetic
    nuSIprop::calculate_flux c2a(3e3, 0.03, 0.1, 2.5, 6, true, true, true, 300, 4, 9, 5, 2, false);
    c2a.evolve();
    dump("D", c2a);
    c2a.set_reference_order(false);            // the opt-in shared-algorithm order
    c2a.evolve();
    dump("E", c2a);
    return 0;
}
