// port_text.cpp — TEST INFRASTRUCTURE ONLY (part of liboracle.so, the CPU "port").
//
// The reference's dist output step, restated for the CPU baseline: CommandDistance::
// writeOutput (CommandDistance.cpp:276-333) streams every passing pair as
//   ref name \t query name \t distance \t p-value \t numer/denom
// through std::cout with the stream's default double formatting (6 significant digits) and
// `endl` (a flush) after every line, on the main thread, in query-major order.  This writes
// the same lines to a file through an std::ofstream (flush per line when flush_each), so the
// bench can time the reference's text step on a sample block of a grid.

#include <cstdint>
#include <fstream>

extern "C" int orc_write_dist_text(const char *path, const char *names, const uint64_t *name_off,
                                   uint32_t n_ref, const uint32_t *qry_rows, uint32_t n_q,
                                   const uint32_t *numer, const uint32_t *denom,
                                   const double *dist, const double *pval, const uint8_t *pass,
                                   int flush_each)
{
    std::ofstream out(path, std::ios::binary | std::ios::trunc);
    if (!out) return -1;
    for (uint32_t i = 0; i < n_q; i++) {
        const uint32_t q = qry_rows[i];
        for (uint32_t j = 0; j < n_ref; j++) {
            const uint64_t c = (uint64_t)i * n_ref + j;
            if (pass && !pass[c]) continue;
            out.write(names + name_off[j], (std::streamsize)(name_off[j + 1] - name_off[j]));
            out << '\t';
            out.write(names + name_off[q], (std::streamsize)(name_off[q + 1] - name_off[q]));
            out << '\t' << dist[c] << '\t' << pval[c] << '\t' << numer[c] << '/' << denom[c];
            if (flush_each) out << std::endl;
            else out << '\n';
        }
    }
    out.flush();
    return out ? 0 : -2;
}
