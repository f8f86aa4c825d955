// bioinfo1_amd/csrc/tm_main.cpp -- team_mapper_amd: the reference mapper's
// command line (team_mapper.cpp:165-180, 319-396) over the MI355X pipeline
// (tm_map_files).  PAF-like lines go to stdout in read order.
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <string>

#include "../../include/team_align_c.h"
#include "../../include/team_mapper_c.h"

#define TM_VERSION "3.1.0"
#define TM_PROGRAM "toolForGenomeAllignment"

static void help() {
    std::printf(
        "\nUsage: %s[options] <file1> <file2>\n"
        "NOTE: file1 needs to be in FASTA format, while the second file will contain a set of fragments in either "
        "FASTA or FASTQ format.\n"
        "Options: \n"
        "\t  -a, --alignment TYPE     Alignment type: global, local, semiGlobal\n"
        "\t  -m MATCH                 Match score (default: 1)\n"
        "\t  -n MISMATCH              Mismatch penalty (default: -1)\n"
        "\t  -g GAP                   Gap penalty (default: -1)\n"
        "\t  -k KMER                  k-mer length for minimizers (default: 15)\n"
        "\t  -w WINDOW                window size for minimizers (default: 5)\n"
        "\t  -f FREQUENCY_THRESHOLD   Frequency threshold factor (default: 0.001)\n"
        "\t  -c                       Output CIGAR string\n"
        "\t  -h, --help               Show this help message\n"
        "\t  --version                Show version information\n"
        "\t  -d DEVICE                GPU index (default: 0)\n",
        TM_PROGRAM);
}

int main(int argc, char** argv) {
    tm_options o{TA_GLOBAL, 1, -1, -1, 15, 5, 0.001, 0, 0};
    std::string f1, f2;
    int device = 0;
    if (argc < 2) {
        std::fprintf(stderr, "Error: Not enough arguments\n");
        help();
        return 1;
    }
    if (!std::strcmp(argv[1], "-h") || !std::strcmp(argv[1], "--help")) {
        help();
        return 0;
    }
    if (!std::strcmp(argv[1], "--version")) {
        std::printf("%s v%s\n", TM_PROGRAM, TM_VERSION);
        return 0;
    }
    if (argc < 3) {
        std::fprintf(stderr, "Error: Expected two input files\n");
        return 1;
    }
    for (int i = 1; i < argc; ++i) {
        const char* a = argv[i];
        const bool more = i + 1 < argc;
        if (!std::strcmp(a, "-a") && more) {
            const char* t = argv[++i];
            if (!std::strcmp(t, "global")) o.type = TA_GLOBAL;
            else if (!std::strcmp(t, "local")) o.type = TA_LOCAL;
            else if (!std::strcmp(t, "semiGlobal")) o.type = TA_SEMI_GLOBAL;
            else {
                std::fprintf(stderr, "Error: Expected Alignment type: global, local, semiGlobal\n");
                help();
                return 1;
            }
        } else if (!std::strcmp(a, "-m") && more) o.match = std::atoi(argv[++i]);
        else if (!std::strcmp(a, "-n") && more) o.mismatch = std::atoi(argv[++i]);
        else if (!std::strcmp(a, "-g") && more) o.gap = std::atoi(argv[++i]);
        else if (!std::strcmp(a, "-k") && more) o.k = (unsigned)std::atoi(argv[++i]);
        else if (!std::strcmp(a, "-w") && more) o.w = (unsigned)std::atoi(argv[++i]);
        else if (!std::strcmp(a, "-f") && more) o.f = std::strtod(argv[++i], nullptr);
        else if (!std::strcmp(a, "-d") && more) device = std::atoi(argv[++i]);
        else if (!std::strcmp(a, "-c")) o.want_cigar = 1;
        else if (!std::strcmp(a, "-s")) std::fprintf(stderr, "note: -s (statistics) is not part of this build\n");
        else if (f1.empty()) f1 = a;
        else if (f2.empty()) f2 = a;
        else {
            std::fprintf(stderr, "Unknown or extra argument: %s\n", a);
            help();
            return 1;
        }
    }
    if (f1.empty() || f2.empty()) {
        std::fprintf(stderr, "Error: Two input files are required.\n");
        help();
        return 1;
    }
    const int r = tm_map_files(f1.c_str(), f2.c_str(), &o, "-", device);
    if (r != TM_OK && r != TM_ERR_INPUT) std::fprintf(stderr, "error: %s\n", tm_status_string(r));
    return r == TM_OK ? 0 : 1;
}
