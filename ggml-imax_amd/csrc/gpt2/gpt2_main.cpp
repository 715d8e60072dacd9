// gpt2_main.cpp -- `gpt-2-mi355x`, the command line of examples/gpt-2/main-backend.cpp:788-945
// (options of examples/common.cpp:42-70, defaults of common.h:19-43) over gpt2-mi355x.h.
//
//   gpt-2-mi355x -m model.bin [-p prompt] [-n n_predict] [-s seed] [-t threads] [-b n_batch]
//                [-c n_ctx] [-ngl N] [--top_k K] [--top_p P] [--temp T] [--ignore-eos]
//
// -ngl > 0 runs the whole graph on MI355X device 0 (the reference picks its GPU backend the same
// way, main-backend.cpp:199-230); -ngl 0 asks the ggml registry for "CPU", which exists when this
// file is linked against the reference libggml (the oracle build).

#include "gpt2-mi355x.h"

#include <dlfcn.h>

#include <algorithm>
#include <cmath>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <ctime>
#include <random>
#include <string>
#include <vector>

namespace {

struct params {
    int32_t seed = -1;
    int32_t n_threads = 4;
    int32_t n_predict = 200;
    int32_t n_batch = 8;
    int32_t n_ctx = 2048;
    int32_t n_gpu_layers = 0;
    bool ignore_eos = false;
    int32_t top_k = 40;
    float top_p = 0.9f;
    float temp = 0.9f;
    std::string model = "models/gpt-2-117M/ggml-model.bin";
    std::string prompt;
};

void usage(const char * argv0) {
    fprintf(stderr,
            "usage: %s -m MODEL [-p PROMPT] [-n N_PREDICT] [-s SEED] [-t THREADS] [-b N_BATCH] [-c N_CTX]\n"
            "          [-ngl N_GPU_LAYERS] [--top_k K] [--top_p P] [--temp T] [--ignore-eos]\n",
            argv0);
}

bool parse(int argc, char ** argv, params & p) {
    for (int i = 1; i < argc; i++) {
        const std::string a = argv[i];
        auto next = [&]() -> const char * {
            if (i + 1 >= argc) {
                fprintf(stderr, "error: missing value for %s\n", a.c_str());
                exit(1);
            }
            return argv[++i];
        };
        if (a == "-s" || a == "--seed") p.seed = atoi(next());
        else if (a == "-t" || a == "--threads") p.n_threads = atoi(next());
        else if (a == "-p" || a == "--prompt") p.prompt = next();
        else if (a == "-n" || a == "--n_predict") p.n_predict = atoi(next());
        else if (a == "-b" || a == "--batch_size") p.n_batch = atoi(next());
        else if (a == "-c" || a == "--context") p.n_ctx = atoi(next());
        else if (a == "-ngl" || a == "--gpu-layers" || a == "--n-gpu-layers") p.n_gpu_layers = atoi(next());
        else if (a == "--top_k") p.top_k = atoi(next());
        else if (a == "--top_p") p.top_p = (float) atof(next());
        else if (a == "--temp") p.temp = (float) atof(next());
        else if (a == "-m" || a == "--model") p.model = next();
        else if (a == "--ignore-eos") p.ignore_eos = true;
        else if (a == "-h" || a == "--help") {
            usage(argv[0]);
            exit(0);
        } else {
            fprintf(stderr, "error: unknown argument: %s\n", a.c_str());
            usage(argv[0]);
            return false;
        }
    }
    return true;
}

// top-k / top-p / temperature sampling with the arithmetic of examples/common.cpp:427-505:
// double logits*1/temp, partial sort of top_k, exp(l - max) / sum, nucleus cut at the first
// cumulative >= top_p, renormalise, std::discrete_distribution on the caller's mt19937.
int32_t sample(const float * logits, int n_vocab, int top_k, double top_p, double temp, std::mt19937 & rng) {
    std::vector<std::pair<double, int32_t>> cand(n_vocab);
    const double scale = 1.0 / temp;
    for (int i = 0; i < n_vocab; i++) cand[i] = {logits[i] * scale, i};
    top_k = std::min(top_k, n_vocab);
    std::partial_sort(cand.begin(), cand.begin() + top_k, cand.end(),
                      [](const std::pair<double, int32_t> & a, const std::pair<double, int32_t> & b) { return a.first > b.first; });
    cand.resize(top_k);
    double maxl = -INFINITY;
    for (const auto & c : cand) maxl = std::max(maxl, c.first);
    std::vector<double> probs;
    probs.reserve(cand.size());
    double sum = 0.0;
    for (const auto & c : cand) {
        const double e = exp(c.first - maxl);
        probs.push_back(e);
        sum += e;
    }
    for (auto & pr : probs) pr /= sum;
    if (top_p < 1.0f) {
        double cum = 0.0f;
        for (int i = 0; i < top_k; i++) {
            cum += probs[i];
            if (cum >= top_p) {
                top_k = i + 1;
                probs.resize(top_k);
                cand.resize(top_k);
                break;
            }
        }
        cum = 1.0 / cum;
        for (auto & pr : probs) pr *= cum;
    }
    std::discrete_distribution<> dist(probs.begin(), probs.end());
    return cand[dist(rng)].second;
}

// one of the reference's canned prompts when -p is absent (examples/common.cpp:132-150 draws from
// a fixed list with the same generator; this list is our own)
std::string random_prompt(std::mt19937 & rng) {
    static const char * k[] = {"So", "Once upon a time", "When", "The", "After", "If", "import", "He", "She", "They"};
    return k[rng() % (sizeof(k) / sizeof(k[0]))];
}

} // namespace

int main(int argc, char ** argv) {
    ggml_time_init();
    const int64_t t_main_start_us = ggml_time_us();
    params p;
    if (!parse(argc, argv, p)) return 1;
    if (p.seed < 0) p.seed = (int32_t) time(nullptr);
    printf("%s: seed = %d\n", __func__, p.seed);
    std::mt19937 rng(p.seed);
    if (p.prompt.empty()) p.prompt = random_prompt(rng);

    const char * want = p.n_gpu_layers > 0 ? "MI355X0" : "CPU";
    ggml_backend_t backend = ggml_backend_reg_init_backend_from_str(want);
    if (!backend) {
        fprintf(stderr, "%s: backend '%s' is not available in this build\n", __func__, want);
        return 1;
    }
    fprintf(stderr, "%s: using %s backend\n", __func__, ggml_backend_name(backend));
    if (strcmp(ggml_backend_name(backend), "CPU") == 0) {
        typedef void (*set_threads_fn)(ggml_backend_t, int);
        if (auto fn = (set_threads_fn) dlsym(RTLD_DEFAULT, "ggml_backend_cpu_set_n_threads")) fn(backend, p.n_threads);
    }

    const int64_t t_load0 = ggml_time_us();
    // on the MI355X backend: inputs read in place from pinned host memory, logits staged through it
    ggml_backend_buffer_type_t host_buft = nullptr;
    typedef ggml_backend_buffer_type_t (*host_buft_fn)(void);
    if (strcmp(ggml_backend_name(backend), "CPU") != 0) {
        if (auto fn = (host_buft_fn) dlsym(RTLD_DEFAULT, "ggml_backend_mi355x_host_buffer_type")) host_buft = fn();
    }
    gpt2_model * model = gpt2_model_load_ex(p.model.c_str(), backend, p.n_ctx, p.n_batch, host_buft);
    if (!model) {
        fprintf(stderr, "%s: failed to load model from '%s'\n", __func__, p.model.c_str());
        ggml_backend_free(backend);
        return 1;
    }
    const int64_t t_load_us = ggml_time_us() - t_load0;
    gpt2_hparams_c hp;
    gpt2_model_hparams(model, &hp);
    printf("%s: model size  = %8.2f MB\n", __func__, gpt2_model_size(model) / 1024.0 / 1024.0);
    fprintf(stderr, "%s: compute buffer size: %.2f MB\n", __func__, gpt2_compute_buffer_size(model) / 1024.0 / 1024.0);

    std::vector<int32_t> inp(4096);
    const int n_inp = gpt2_tokenize(model, p.prompt.c_str(), inp.data(), (int) inp.size());
    inp.resize(std::min<int>(n_inp, (int) inp.size()));
    p.n_predict = std::min(p.n_predict, hp.n_ctx - (int) inp.size());
    printf("%s: prompt: '%s'\n", __func__, p.prompt.c_str());
    printf("%s: number of tokens in prompt = %zu, first 8 tokens: ", __func__, inp.size());
    for (int i = 0; i < std::min(8, (int) inp.size()); i++) printf("%d ", inp[i]);
    printf("\n\n");

    int n_past = 0;
    int64_t t_sample_us = 0, t_predict_us = 0;
    std::vector<float> logits(hp.n_vocab);
    std::vector<int32_t> embd;
    for (size_t i = 0; i < inp.size() + (size_t) p.n_predict; i++) {
        if (!embd.empty()) {
            const int64_t t0 = ggml_time_us();
            if (gpt2_eval(model, n_past, embd.data(), (int) embd.size(), logits.data(), 0) != 0) {
                printf("Failed to predict\n");
                return 1;
            }
            t_predict_us += ggml_time_us() - t0;
        }
        n_past += (int) embd.size();
        embd.clear();
        if (i >= inp.size()) {
            const int64_t t0 = ggml_time_us();
            embd.push_back(sample(logits.data(), hp.n_vocab, p.top_k, p.top_p, p.temp, rng));
            t_sample_us += ggml_time_us() - t0;
        } else {
            for (size_t k = i; k < inp.size(); k++) {
                embd.push_back(inp[k]);
                if ((int32_t) embd.size() >= p.n_batch) break;
            }
            i += embd.size() - 1;
        }
        for (int32_t id : embd) printf("%s", gpt2_token_text(model, id));
        fflush(stdout);
        if (!p.ignore_eos && embd.back() == 50256) break;
    }

    const int64_t t_main_end_us = ggml_time_us();
    printf("\n\n");
    printf("%s:     load time = %8.2f ms\n", __func__, t_load_us / 1000.0f);
    printf("%s:   sample time = %8.2f ms\n", __func__, t_sample_us / 1000.0f);
    printf("%s:  predict time = %8.2f ms / %.2f ms per token\n", __func__, t_predict_us / 1000.0f,
           t_predict_us / 1000.0f / std::max(n_past, 1));
    printf("%s:    total time = %8.2f ms\n", __func__, (t_main_end_us - t_main_start_us) / 1000.0f);

    gpt2_model_free(model);
    ggml_backend_free(backend);
    return 0;
}
