// nuSIprop.hpp -- C++ drop-in facade over the MI355X C ABI (include/nusi.h).
//
// Same class, constructors, public members, methods and error behaviour as
// the reference's nuSIprop::calculate_flux (nuSIprop.hpp:22-540); the work is
// done by libnusi.so on the GPU.  Link with -L<repo>/nusiprop_amd -lnusi.
//
//   reference                                  here
//   calculate_flux()            :59            same defaults (1e7, 0.1, 0.1, 2, 1, true, false)
//   calculate_flux(mphi, ...)   :61-65         same argument list and defaults
//   public mphi g mntot si norm :174           re-read by every evolve()
//   evolve()                    :176-337       nusi_set_params + nusi_evolve
//   check_energy_conservation() :339-357       nusi_check_energy_conservation
//   get_flux / get_flux_fla     :359-405       same range messages on stderr, 0 returned
//   get_N_bins_E / get_energy   :407-429
//   copy ctor / operator= / dtor :434-540      deep copy (nusi_copy)
//
// Fatal conditions the reference ends with exit(1) (no mass spectrum,
// aux.hpp:48; missing phi-phi tables, interp.hpp:251-254; out-of-range
// phi-phi lookup, interp.hpp:355-361) print the library's message and exit(1)
// here too; so does a HIP error (no GPU).  Negative cross sections print a
// warning on stderr and continue, as in the reference (:909-918, :1215-1231,
// :1505-1516).  Deliberate difference: the reference's getters read one past
// the end for j == N_bins_E (:374, :398, :422: the test is j > N_bins_E);
// here that index returns 0 without reading out of bounds.  check_energy_conservation()
// before any evolve() returns NaN with a message (the reference reads an uninitialised
// norm_total there, nuSIprop.hpp:341).
#ifndef NUSIPROP_MI355X_HPP
#define NUSIPROP_MI355X_HPP

#include <cstdlib>
#include <iostream>
#include <vector>

#include "nusi.h"

namespace nuSIprop {

class calculate_flux {
public:
    calculate_flux() : calculate_flux(1e7, 0.1, 0.1, 2, 1, true, false) {}

    calculate_flux(double mphi_, double g_, double mntot_, double si_, double norm_ = 1, bool majorana_ = true,
                   bool non_resonant_ = true, bool normal_ordering_ = true, int N_bins_E_ = 300, double lEmin_ = 12.0,
                   double lEmax_ = 17.0, double zmax_ = 5.0, int flav_ = 2, bool phiphi_ = false)
        : mphi(mphi_), g(g_), mntot(mntot_), si(si_), norm(norm_)
    {
        nusi_params p;
        nusi_params_default(&p, mphi_, g_, mntot_, si_);
        p.norm = norm_;
        p.majorana = majorana_;
        p.non_resonant = non_resonant_;
        p.normal_ordering = normal_ordering_;
        p.N_bins_E = N_bins_E_;
        p.lEmin = lEmin_;
        p.lEmax = lEmax_;
        p.zmax = zmax_;
        p.flav = flav_;
        p.phiphi = phiphi_;
        p.source_model = NUSI_SOURCE_DSNB;
        check(nusi_create(&p, &h_));
        init_buffers();
    }

    calculate_flux(const calculate_flux& o) : mphi(o.mphi), g(o.g), mntot(o.mntot), si(o.si), norm(o.norm)
    {
        check(nusi_copy(o.h_, &h_));
        init_buffers();
        flux_ = o.flux_;
        flux_fla_ = o.flux_fla_;
    }

    calculate_flux& operator=(const calculate_flux& o)
    {
        if (this != &o) {
            nusi_handle* h = nullptr;
            check(nusi_copy(o.h_, &h));
            nusi_destroy(h_);
            h_ = h;
            mphi = o.mphi;
            g = o.g;
            mntot = o.mntot;
            si = o.si;
            norm = o.norm;
            init_buffers();
            flux_ = o.flux_;
            flux_fla_ = o.flux_fla_;
        }
        return *this;
    }

    ~calculate_flux() { nusi_destroy(h_); }

    // Parameters that may be changed between runs (reference :174)
    double mphi, g, mntot, si, norm;

    void evolve(void)
    {
        check(nusi_set_params(h_, mphi, g, mntot, si, norm));
        check(nusi_evolve(h_));
        fetch();
    }

    double check_energy_conservation(void)
    {
        double r = 0;
        check(nusi_set_params(h_, mphi, g, mntot, si, norm));
        const int e = nusi_check_energy_conservation(h_, &r);
        if (e == NUSI_ESTATE)   // before any evolve(): the reference reads norm_total uninitialised; NaN + message
            std::cerr << nusi_last_error() << std::endl;
        else
            check(e);
        fetch();
        return r;
    }

    double get_flux(int i, int j)
    {
        if (i < 0 || i >= 3) {
            std::cerr << "You asked for the flux of the mass eigenstate " << i << ", not in [0,1,2]. Zero will be returned."
                      << std::endl;
            return 0;
        }
        if (!bin_ok(j)) return 0;
        return j < N_ ? flux_[(size_t)i * N_ + j] : 0.0;
    }

    double get_flux_fla(int i, int j)
    {
        if (i < 0 || i >= 3) {
            std::cerr << "You asked for the flux of the flavor eigenstate " << i << ", not in [0,1,2]. Zero will be returned."
                      << std::endl;
            return 0;
        }
        if (!bin_ok(j)) return 0;
        return j < N_ ? flux_fla_[(size_t)i * N_ + j] : 0.0;
    }

    int get_N_bins_E(void) { return N_; }

    double get_energy(int i)
    {
        if (i < 0) {
            std::cerr << "You asked for the energy at the bin " << i << "<0! Zero will be returned." << std::endl;
            return 0;
        }
        if (i > N_) {
            std::cerr << "You asked for the energy at the bin " << i << ", but there are only " << N_
                      << " bins! Zero will be returned." << std::endl;
            return 0;
        }
        return i < N_ ? E_[i] : 0.0;
    }

    // extension (no reference counterpart): true (the default) = evolve() builds the tables in the reference's own
    // dilogarithm arithmetic (NUSI_OPT_REFERENCE_ORDER, include/nusi.h); false = the opt-in shared-algorithm order
    // (faster; up to ~1e-6 from the reference's fluxes where its closed forms cancel); kept by copies
    void set_reference_order(bool on) { check(nusi_set_option(h_, NUSI_OPT_REFERENCE_ORDER, on ? 1 : 0)); }

private:
    nusi_handle* h_ = nullptr;
    int N_ = 0;
    std::vector<double> E_, flux_, flux_fla_;

    static void check(int r)
    {
        if (r != NUSI_OK) {
            std::cerr << nusi_last_error() << std::endl;
            std::exit(1);
        }
    }

    bool bin_ok(int j) const
    {
        if (j < 0) {
            std::cerr << "You asked for the flux at the energy bin " << j << "<0! Zero will be returned." << std::endl;
            return false;
        }
        if (j > N_) {
            std::cerr << "You asked for the flux at the energy bin " << j << ", but there are only " << N_
                      << " bins! Zero will be returned." << std::endl;
            return false;
        }
        return true;
    }

    void init_buffers()
    {
        N_ = nusi_get_N_bins_E(h_);
        E_.assign(N_, 0.0);
        flux_.assign(3 * (size_t)N_, 0.0);
        flux_fla_.assign(3 * (size_t)N_, 0.0);
        check(nusi_get_energies(h_, E_.data()));
    }

    void fetch()
    {
        check(nusi_get_flux(h_, flux_.data()));
        check(nusi_get_flux_fla(h_, flux_fla_.data()));
        const int w = nusi_get_warnings(h_);
        static const char* what[3] = {"Gamma", "alphaTilde", "alpha"};
        for (int k = 0; k < 3; ++k)
            if (w & (1 << k))
                std::cerr << "Negative cross section when computing " << what[k] << ". Possible roundoff errors for g="
                          << g << ", mphi=" << mphi << ", mntot=" << mntot << std::endl;
    }
};

}  // namespace nuSIprop

#endif
