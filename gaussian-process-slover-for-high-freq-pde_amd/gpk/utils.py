"""Result-log helpers with the reference's paths, names and formats (code/utils.py:550-619).

Plotting and the pickle re-loaders of the reference (code/utils.py:25-547, :622-837) are out of
scope.  Pickles written here hold plain NumPy arrays and Python objects.
"""
import os
import pickle


def get_prefix(model, trick_paras):
    """result_log/<equation>/kernel_<K>[-extra-<K2>]/epoch_<n>/Q<Q>/ (utils.py:550-568)."""
    if trick_paras.get("kernel_extra") is not None:
        prefix = "result_log/" + trick_paras["equation"] + "/kernel_" + \
            model.cov_func.__class__.__name__ + "-extra-" + model.cov_func_extra.__class__.__name__ + \
            "/epoch_" + str(trick_paras["nepoch"]) + "/Q" + str(trick_paras["Q"]) + "/"
    else:
        prefix = "result_log/" + trick_paras["equation"] + "/kernel_" + \
            model.cov_func.__class__.__name__ + "/epoch_" + str(trick_paras["nepoch"]) + \
            "/Q" + str(trick_paras["Q"]) + "/"
    if not os.path.exists(prefix):
        os.makedirs(prefix)
    return prefix


def get_save_name(trick_paras):
    """utils.py:571-577."""
    return "llk_weight-%.1f-nu-%d-Q-%d-epoch-%d-lr-%.4f-freqscale=%d-logdet-%d" % (
        trick_paras["llk_weight"], trick_paras["num_u_trick"], trick_paras["Q"],
        trick_paras["nepoch"], trick_paras["lr"], trick_paras["freq_scale"],
        trick_paras["logdet"]) + trick_paras["other_paras"]


def store_model(model, log_dict, trick_paras):
    """pickle (params, log_dict, trick_paras) (utils.py:580-597)."""
    prefix = get_prefix(model, trick_paras)
    save_name = get_save_name(trick_paras)
    params = model.params
    if trick_paras.get("kernel_extra") is not None:
        data = (params, model.params_extra, log_dict, trick_paras)
    else:
        data = (params, log_dict, trick_paras)
    with open(prefix + save_name + ".pkl", "wb") as f:
        pickle.dump(data, f)
    print("save model, log_dict, trick_paras to ", prefix + save_name + ".pkl")


def wrirte_log(model, err_dict, trick_paras):
    """Append the run summary to log.txt (utils.py:600-619; the name's typo is the reference's)."""
    prefix = get_prefix(model, trick_paras)
    with open(prefix + "log.txt", "a+") as f:
        f.write("llk_weight-%.1f--nu-%d-Q-%d-epoch-%d-lr-%.4f-freqscale=%d-logdet-%d" % (
            trick_paras["llk_weight"], trick_paras["num_u_trick"], trick_paras["Q"],
            trick_paras["nepoch"], trick_paras["lr"], trick_paras["freq_scale"],
            trick_paras["logdet"]) + trick_paras["other_paras"] + "\n")
        f.write("err_mean: %.4f, err_std: %.4f, used_time: %.4f, avg_time: %.4f, avg_epochs %d \n" % (
            err_dict["mean"], err_dict["std"], err_dict["used_time"], err_dict["avg_time"],
            err_dict["stop_epoch_mean"]))
        f.write("err_list: " + str(err_dict["err_list"]) + "\n\n\n")
    print("write log to ", prefix + "log.txt")
