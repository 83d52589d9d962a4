// lt_load_check.cpp -- checkpoint-compatibility harness (test tool, linked against libtorch).
//
// Builds the reference's model the way GGL::Model's constructor does (Models.cpp:7-33: per hidden
// layer Linear, LayerNorm if enabled, the activation; then the output Linear -- none when out is 0,
// the shared head's addOutputLayer = false, Models.cpp:24-28), loads a <NAME>.lt
// file with torch::load(seq, stream) as Model::Load does (Models.cpp:130-166, including its
// parameter-size check), runs the float forward on the rows of an input file and writes the
// outputs -- or, with "save", writes the module with torch::save(seq, stream) (Models.cpp:116-120)
// after filling it from a raw parameter file.
//
// usage: lt_load_check load <model.lt> <in.f32> <rows> <out.f32> <obs> <out> <ln 0|1> <h1> [h2 ...]
//        lt_load_check save <params.f32> <model.lt> <obs> <out> <ln 0|1> <h1> [h2 ...]
//        lt_load_check optim <NAME_OPTIM.lt> <dump.bin> <steps> <obs> <out> <ln 0|1> <h1> [h2 ...]
// optim: an AdamW over the model's parameters (Models.h:40-56) takes <steps> steps on a seeded loss,
// then Model::Save's optimizer branch writes the archive (Models.cpp:122-125); dump.bin gets the
// step (int64) and every parameter's exp_avg, then exp_avg_sq, in parameters() order.
#include <torch/torch.h>

#include <cstdio>
#include <fstream>
#include <iostream>
#include <string>
#include <vector>

static torch::nn::Sequential make_model(int obs, int out, bool ln, const std::vector<int>& layers) {
    torch::nn::Sequential seq;
    int last = obs;
    for (int h : layers) {
        seq->push_back(torch::nn::Linear(last, h));
        if (ln) seq->push_back(torch::nn::LayerNorm(torch::nn::LayerNormOptions({(int64_t)h})));
        last = h;
        seq->push_back(torch::nn::LeakyReLU());
    }
    if (out > 0) seq->push_back(torch::nn::Linear(last, out));
    return seq;
}

static std::vector<uint64_t> seq_sizes(torch::nn::Sequential& seq) {
    std::vector<uint64_t> r;
    for (size_t i = 0; i < seq->size(); i++)
        for (auto& p : seq[i]->parameters()) r.push_back(p.numel());
    return r;
}

int main(int argc, char** argv) {
    if (argc < 2) return 2;
    std::string mode = argv[1];
    bool load = mode == "load";
    int a = load ? 6 : (mode == "optim" ? 5 : 4);
    if (argc < a + 4) return 2;
    int obs = std::atoi(argv[a]), out = std::atoi(argv[a + 1]);
    bool ln = std::atoi(argv[a + 2]) != 0;
    std::vector<int> layers;
    for (int i = a + 3; i < argc; i++) layers.push_back(std::atoi(argv[i]));
    torch::nn::Sequential seq = make_model(obs, out, ln, layers);
    if (mode == "optim") {
        torch::manual_seed(5);
        torch::optim::AdamW opt(seq->parameters(), torch::optim::AdamWOptions(2.5e-4));
        for (int k = 0; k < std::atoi(argv[4]); k++) {
            auto loss = seq->forward(torch::randn({8, obs})).square().sum();
            opt.zero_grad();
            loss.backward();
            opt.step();
        }
        torch::serialize::OutputArchive ar;
        opt.save(ar);
        ar.save_to(argv[2]);
        std::vector<float> m, v;
        int64_t step = 0;
        for (auto& p : seq->parameters()) {
            auto& st = static_cast<torch::optim::AdamWParamState&>(*opt.state().at(p.unsafeGetTensorImpl()));
            step = st.step();
            auto a_ = st.exp_avg().contiguous(), b_ = st.exp_avg_sq().contiguous();
            m.insert(m.end(), a_.data_ptr<float>(), a_.data_ptr<float>() + a_.numel());
            v.insert(v.end(), b_.data_ptr<float>(), b_.data_ptr<float>() + b_.numel());
        }
        FILE* g = std::fopen(argv[3], "wb");
        std::fwrite(&step, 8, 1, g);
        std::fwrite(m.data(), 4, m.size(), g);
        std::fwrite(v.data(), 4, v.size(), g);
        std::fclose(g);
        return 0;
    }
    if (load) {
        auto before = seq_sizes(seq);
        std::ifstream in(argv[2], std::ios::binary);
        in >> std::noskipws;
        torch::load(seq, in);
        if (seq_sizes(seq) != before) {
            std::cerr << "Saved model has different size than current model\n";
            return 3;
        }
        int rows = std::atoi(argv[4]);
        std::vector<float> x((size_t)rows * obs);
        FILE* f = std::fopen(argv[3], "rb");
        if (!f || std::fread(x.data(), 4, x.size(), f) != x.size()) return 4;
        std::fclose(f);
        torch::NoGradGuard ng;
        auto y = seq->forward(torch::from_blob(x.data(), {rows, obs})).contiguous();
        FILE* g = std::fopen(argv[5], "wb");
        std::fwrite(y.data_ptr<float>(), 4, (size_t)y.numel(), g);
        std::fclose(g);
    } else {
        std::vector<float> p;
        FILE* f = std::fopen(argv[2], "rb");
        if (!f) return 4;
        float v;
        while (std::fread(&v, 4, 1, f) == 1) p.push_back(v);
        std::fclose(f);
        size_t o = 0;
        torch::NoGradGuard ng;
        for (auto& t : seq->parameters()) {
            if (o + t.numel() > p.size()) return 5;
            t.copy_(torch::from_blob(p.data() + o, t.sizes()));
            o += t.numel();
        }
        std::ofstream os(argv[3], std::ios::binary);
        torch::save(seq, os);
    }
    return 0;
}
