/* phiphi_text_to_binary -- phi-phi table text -> the binary layout the loaders read.
 *
 * Replaces the reference's xsec/text_to_binary.cpp:6-78, which converts
 * xsec/tables_phiphi.py's output (alpha_phiphi.dat: 4 columns, alphatilde_phiphi.dat:
 * 3 columns) into float32 records {x0, .., x_{d-1}, f} written back to back
 * (the layout of interp.hpp:249-291).  Same parsing as the reference: lines
 * starting with '#' are skipped, fields are separated by blanks and each is
 * converted as scanf("%f") does (strtof, round to nearest float).
 *
 * Differences by design: the input is streamed (the reference holds all
 * 100 M records, 1.6 GB, in memory), file names and the field count are
 * arguments, and a short file, a malformed line or a record count other than
 * the expected one is an error (the reference reads a fixed line count and
 * re-uses its last line when the file is short).
 *
 *   phiphi_text_to_binary <in.dat> <out.bin> <fields: 3|4> [expected_records]
 * exit status 0 = ok, 1 = usage / I/O / format error (message on stderr).
 */
#include <errno.h>
#include <stdio.h>
#include <stdlib.h>
#include <string.h>

int main(int argc, char** argv)
{
    if (argc < 4 || argc > 5) {
        fprintf(stderr, "usage: %s <in.dat> <out.bin> <fields: 3|4> [expected_records]\n", argv[0]);
        return 1;
    }
    const int nf = atoi(argv[3]);
    if (nf < 2 || nf > 8) {
        fprintf(stderr, "fields must be in [2, 8] (alphatilde: 3, alpha: 4), got %s\n", argv[3]);
        return 1;
    }
    const long long expect = argc == 5 ? atoll(argv[4]) : -1;
    FILE* in = fopen(argv[1], "r");
    if (!in) {
        fprintf(stderr, "cannot open %s: %s\n", argv[1], strerror(errno));
        return 1;
    }
    FILE* out = fopen(argv[2], "wb");
    if (!out) {
        fprintf(stderr, "cannot create %s: %s\n", argv[2], strerror(errno));
        fclose(in);
        return 1;
    }
    char line[1024];
    float buf[4096 * 8];
    int nbuf = 0;
    long long nrec = 0, lineno = 0;
    int rc = 0;
    while (fgets(line, sizeof line, in)) {
        ++lineno;
        if (line[0] == '#') continue;
        if (!strchr(line, '\n') && !feof(in)) {
            fprintf(stderr, "%s:%lld: line longer than %zu bytes\n", argv[1], lineno, sizeof line - 1);
            rc = 1;
            break;
        }
        const char* p = line;
        int k = 0;
        for (; k < nf; ++k) {
            char* end;
            errno = 0;
            const float v = strtof(p, &end);   /* what sscanf("%f") computes */
            if (end == p) break;
            buf[nbuf * nf + k] = v;
            p = end;
        }
        while (*p == ' ' || *p == '\t' || *p == '\r' || *p == '\n') ++p;
        if (k == 0 && *p == '\0') continue;   /* blank line */
        if (k != nf || *p != '\0') {
            fprintf(stderr, "%s:%lld: expected %d numeric fields\n", argv[1], lineno, nf);
            rc = 1;
            break;
        }
        ++nrec;
        if (++nbuf == 4096) {
            if (fwrite(buf, sizeof(float) * nf, nbuf, out) != (size_t)nbuf) { rc = 1; break; }
            nbuf = 0;
        }
    }
    if (!rc && nbuf && fwrite(buf, sizeof(float) * nf, nbuf, out) != (size_t)nbuf) rc = 1;
    if (ferror(in)) rc = 1;
    if (fclose(out) != 0) rc = 1;
    fclose(in);
    if (!rc && expect >= 0 && nrec != expect) {
        fprintf(stderr, "%s: %lld records, expected %lld\n", argv[1], nrec, expect);
        rc = 1;
    }
    if (rc) {
        remove(argv[2]);
        return 1;
    }
    printf("%lld records of %d float32 -> %s\n", nrec, nf, argv[2]);
    return 0;
}
