// lime-submit -- command surface of bin/lime-submit + LimeMain over the
// MI355X engine.  Usage (bin/lime-submit:7-23, LimeMain.scala:30-57):
//
//   lime-submit [<spark-args> --] <command> <args> [-version]
//
//   intersect A.bed B.bed       cli/Intersection.scala:99-112 (keys stranded)
//   merge     A.bed             cli/Merge.scala:36-44
//   complement A.bed genome.txt cli/Complement.scala:154-166 (prints regions)
//   subtract  A.bed B.bed       DistributedSubtract (API-only in the reference)
//   sort      A.bed             cli/Sort.scala:34-38 (device radix sort)
//   cluster   A.bed             cli/Cluster.scala:36-44 (UnstrandedCluster; the
//                               reference defines it but LimeMain does not
//                               register it)
//   window    A.bed B.bed [-distance D]   cli/Window.scala:42-55 (keys stranded,
//                               DistributedWindow default distance 1000)
//   closest   A.bed B.bed       cli/Closest.scala:45-58 (keys stranded,
//                               SingleClosest)
//
// Everything before "--" is accepted and ignored (there is no Spark).
// Output is one region per line, tab-separated (chrom, start, end), followed
// by the BED name fields of the contributing rows; the reference printed
// Scala tuple toString()s of ADAM Features, which have no stable text form.
#include <stdio.h>
#include <string.h>

#include <string>
#include <vector>

#include "lime_amd.hpp"

using namespace lime;

namespace {

struct Cmd {
    const char *name, *desc;
};
const Cmd kCommands[] = {
    {"complement", "Extract intervals not represented by an interval file."},
    {"intersect", "Compute intersection of regions between two inputs"},
    {"merge", "Merges the regions in a single input"},
    {"subtract", "Remove regions of the second input from the first"},
    {"sort", "Sorts the regions in a single input"},
    {"window", "Compute nearby regions between two inputs"},
    {"cluster", "Cluster (but don't merge) overlapping/nearby intervals"},
    {"closest", "Find the closest region in the second input for each region of the first"},
};

void usage() {
    printf("\nUsage: lime-submit [<spark-args> --] <lime-args> [-version]\n\n");
    printf("Choose one of the following commands:\n\n");
    for (auto &c : kCommands) printf("%20s : %s\n", c.name, c.desc);
    printf("\n");
}

Strand strand_of(int8_t s) {
    return s == 1 ? Strand::Forward : s == 2 ? Strand::Reverse : s == 3 ? Strand::Unknown
                                                                        : Strand::Independent;
}

// BED -> keyed RDD: the text is parsed on the device (lime_bed_parse_device,
// the sc.loadBed replacement); records and names come back to the host
// because the operator mirror keys host-side payloads.
RDD<std::string> load_bed(const std::string &path, bool stranded) {
    std::string text;
    {
        FILE *f = fopen(path.c_str(), "rb");
        if (!f) throw Error(LIME_ERR_IO, "cannot read " + path);
        char buf[1 << 16];
        size_t k;
        while ((k = fread(buf, 1, sizeof(buf), f)) > 0) text.append(buf, k);
        fclose(f);
    }
    lime_dbed *b = nullptr;
    check(lime_bed_parse_device(Engine::thread_default().ctx(), text.data(),
                                (int64_t)text.size(), &b));
    const int64_t n = lime_dbed_rows(b);
    std::vector<int32_t> c((size_t)n), nl((size_t)n);
    std::vector<int64_t> s((size_t)n), e((size_t)n), no((size_t)n);
    std::vector<int8_t> st((size_t)n);
    int rc = lime_dbed_fill_host(b, c.data(), s.data(), e.data(), st.data(), no.data(), nl.data());
    std::vector<std::string> names;
    for (int32_t i = 0; i < lime_dbed_contigs(b); ++i) names.push_back(lime_dbed_contig_name(b, i));
    lime_dbed_free(b);
    check(rc);
    RDD<std::string> rdd;
    rdd.reserve((size_t)n);
    for (int64_t i = 0; i < n; ++i)
        rdd.push_back({ReferenceRegion(names[c[i]], s[i], e[i],
                                       stranded ? strand_of(st[i]) : Strand::Independent),
                       text.substr((size_t)no[i], (size_t)nl[i])});
    return rdd;
}

void print_region(const ReferenceRegion &r) {
    printf("%s\t%lld\t%lld", r.referenceName.c_str(), (long long)r.start, (long long)r.end);
}

int run(const std::vector<std::string> &args) {
    const std::string &cmd = args[0];
    auto need = [&](size_t k) {
        if (args.size() < k + 1) throw Error(LIME_ERR_ARG, cmd + ": expected " + std::to_string(k) + " arguments");
    };
    if (cmd == "intersect") {
        need(2);
        auto out = DistributedIntersection<std::string, std::string>(load_bed(args[1], true),
                                                                     load_bed(args[2], true))
                       .compute();
        for (auto &o : out) {
            print_region(o.first);
            printf("\t%s\t%s\n", o.second.first.c_str(), o.second.second.c_str());
        }
    } else if (cmd == "cluster") {
        need(1);
        auto out = UnstrandedCluster<std::string>(load_bed(args[1], true)).compute();
        for (auto &o : out) {
            print_region(o.first);
            printf("\t%zu", o.second.size());
            for (auto &v : o.second) printf("\t%s", v.c_str());
            printf("\n");
        }
    } else if (cmd == "window") {
        need(2);
        int64_t d = 1000;
        for (size_t i = 3; i + 1 < args.size(); ++i)
            if (args[i] == "-distance") d = std::stoll(args[i + 1]);
        auto out = DistributedWindow<std::string, std::string>(load_bed(args[1], true),
                                                               load_bed(args[2], true), {}, d)
                       .compute();
        for (auto &o : out) {
            print_region(o.first);
            printf("\t%s\t%s\n", o.second.first.c_str(), o.second.second.c_str());
        }
    } else if (cmd == "closest") {
        need(2);
        auto out = SingleClosest<std::string, std::string>(load_bed(args[1], true),
                                                           load_bed(args[2], true))
                       .compute();
        for (auto &o : out) {
            print_region(o.first);
            printf("\t%s\t%s\n", o.second.first.c_str(), o.second.second.c_str());
        }
    } else if (cmd == "subtract") {
        need(2);
        auto out = DistributedSubtract<std::string, std::string>(load_bed(args[1], true),
                                                                 load_bed(args[2], true))
                       .compute();
        for (auto &o : out) {
            print_region(o.first);
            printf("\t%s\t%s\n", o.second.first.c_str(),
                   o.second.second ? o.second.second->c_str() : ".");
        }
    } else if (cmd == "merge") {
        need(1);
        auto out = DistributedMerge<std::string>(load_bed(args[1], true)).compute();
        for (auto &o : out) {
            print_region(o.first);
            printf("\t%zu\n", o.second.size());
        }
    } else if (cmd == "complement") {
        need(2);
        int32_t n = 0;
        char **names = nullptr;
        int64_t *lens = nullptr;
        check(lime_genome_read(args[2].c_str(), &n, &names, &lens));
        std::map<std::string, ReferenceRegion> bounds;
        for (int32_t i = 0; i < n; ++i) bounds[names[i]] = ReferenceRegion(names[i], 0, lens[i]);
        lime_genome_free(n, names, lens);
        auto out = DistributedComplement<std::string>(load_bed(args[1], false), {}, bounds).compute();
        for (auto &o : out) {
            print_region(o.first);
            printf("\n");
        }
    } else if (cmd == "sort") {
        need(1);
        auto rdd = load_bed(args[1], true);
        // a merge-free pass through the device sort: runs of a set keyed by
        // its own rows give the canonical order
        std::map<std::string, int64_t> ext;
        for (auto &kv : rdd) ext[kv.first.referenceName] = std::max(ext[kv.first.referenceName], kv.first.end);
        std::vector<std::string> nm;
        std::vector<int64_t> ln;
        for (auto &kv : ext) {
            nm.push_back(kv.first);
            ln.push_back(kv.second);
        }
        // (a genome past 2^32 bases: one space after the other, in order)
        detail::Genome gn(nm, ln);
        auto parts = gn.split(rdd, detail::all_rows(rdd.size()));
        std::vector<size_t> order;
        for (size_t q = 0; q < gn.spaces.size(); ++q) {
            const auto &rows = parts[q];
            if (rows.empty()) continue;
            detail::SetHandle A;
            detail::upload(Engine::thread_default().ctx(), *gn.spaces[q], rdd, rows, A);
            const size_t m = rows.size();
            std::vector<int32_t> c(m);
            std::vector<int64_t> s(m), e(m), r(m);
            check(lime_set_fill_host(A.h, c.data(), s.data(), e.data(), r.data()));
            // the device order ties equal starts by (zero-width first, input
            // row); RegionOrdering ties by end: re-order each (tiny) group
            for (size_t i = 0; i < m;) {
                size_t j = i + 1;
                while (j < m && c[j] == c[i] && s[j] == s[i]) ++j;
                if (j - i > 1)
                    std::stable_sort(r.begin() + i, r.begin() + j, [&](int64_t x, int64_t y) {
                        return rdd[rows[x]].first.end < rdd[rows[y]].first.end;
                    });
                i = j;
            }
            for (size_t i = 0; i < m; ++i) order.push_back(rows[r[i]]);
        }
        for (size_t i : order) {
            print_region(rdd[i].first);
            printf("\t%s\n", rdd[i].second.c_str());
        }
    } else {
        usage();
    }
    return 0;
}

}  // namespace

int main(int argc, char **argv) {
    std::vector<std::string> all(argv + 1, argv + argc), lime_args;
    // bin/lime-submit:7-23: everything after the first "--" is for lime
    auto dd = std::find(all.begin(), all.end(), std::string("--"));
    if (dd != all.end())
        lime_args.assign(dd + 1, all.end());
    else
        lime_args = all;
    bool version = false;
    std::vector<std::string> rest;
    for (auto &a : lime_args) {
        if (a == "-version")
            version = true;
        else
            rest.push_back(a);
    }
    if (version) printf("Version 0\n");  // LimeMain.scala:20-22
    if (rest.empty()) {
        usage();
        return 0;
    }
    bool known = false;
    for (auto &c : kCommands) known |= rest[0] == c.name;
    if (!known) {
        usage();
        return 0;
    }
    try {
        return run(rest);
    } catch (const NoSuchElement &e) {
        fprintf(stderr, "java.util.NoSuchElementException: %s\n", e.what());
        return 1;
    } catch (const Error &e) {
        fprintf(stderr, "lime-submit: %s (status %d)\n", e.what(), e.code);
        return 1;
    }
}
