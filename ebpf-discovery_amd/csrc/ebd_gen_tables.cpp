// ebd_gen_tables.cpp — integer CDF tables for the synthetic trace generator.
//
// Built with +, -, *, / and exact scaling only (own exp/log series), so every host
// produces the same bytes and CPU / GPU traces match everywhere.
#include <cmath>
#include <vector>

#include "ebd_gen.h"

namespace ebd {

namespace {

double exp_det(double x) {
	// x = k*ln2 + r, |r| <= ln2/2; exp(r) by Taylor series; 2^k exactly.
	const double ln2 = 0.69314718055994530942;
	double kf = x / ln2;
	long k = (long)(kf < 0 ? kf - 0.5 : kf + 0.5);
	double r = x - (double)k * ln2;
	double term = 1.0, sum = 1.0;
	for (int i = 1; i < 30; i++) {
		term = term * r / (double)i;
		sum += term;
	}
	return std::ldexp(sum, (int)k);
}

double log_det(double x) {
	// x = m * 2^e, m in [1, 2): ln m = 2 atanh((m-1)/(m+1)).
	int e;
	double m = std::frexp(x, &e) * 2.0;
	e -= 1;
	double t = (m - 1.0) / (m + 1.0), t2 = t * t, term = t, sum = 0.0;
	for (int i = 1; i < 80; i += 2) {
		sum += term / (double)i;
		term *= t2;
	}
	return 2.0 * sum + (double)e * 0.69314718055994530942;
}

void to_cdf(const std::vector<double>& w, uint32_t* out) {
	double total = 0.0;
	for (double v : w)
		total += v;
	double acc = 0.0;
	for (size_t k = 0; k < w.size(); k++) {
		acc += w[k];
		double f = acc / total;
		if (f > 1.0)
			f = 1.0;
		double t = f * 4294967295.0;
		out[k] = (uint32_t)t;
	}
	out[w.size() - 1] = 0xffffffffu;
}

} // namespace

// Lengths: lognormal(mu = ln 205, sigma = 0.62) folded into [32, 1024] (mean ~ 256 B
// after the minimum request size lifts the short tail); Zipf(s = 1.1) for paths and hosts.
void build_gen_tables(GenTables* T) {
	const double mu = log_det(205.0), sigma = 0.62;
	std::vector<double> lw(kLenN, 0.0);
	for (uint32_t L = 1; L <= 20000; L++) {
		const double z = (log_det((double)L) - mu) / sigma;
		const double w = exp_det(-0.5 * z * z) / (double)L;
		uint32_t c = L < kLenMin ? kLenMin : (L > kLenMax ? kLenMax : L);
		lw[c - kLenMin] += w;
	}
	to_cdf(lw, T->len_cdf);
	std::vector<double> hw(kHosts), pw(kPaths);
	for (uint32_t k = 0; k < kHosts; k++)
		hw[k] = exp_det(-1.1 * log_det((double)(k + 1)));
	for (uint32_t k = 0; k < kPaths; k++)
		pw[k] = exp_det(-1.1 * log_det((double)(k + 1)));
	to_cdf(hw, T->host_cdf);
	to_cdf(pw, T->path_cdf);
}

} // namespace ebd
