"""Evaluation metrics of the regressor — mirror of `/root/reference/losses.py:276-366`.

These run on the host (numpy + scikit-learn) exactly as in the reference: they
are O(N) bookkeeping on a few hundred predictions, after the device work
(SURVEY.md §8a a12).  The reference's quirks are kept: the weighted F1 passes
(y_pred, y_true) swapped (losses.py:291), and POM values are rounded lists.

The latent-optimisation likelihoods of losses.py:13-274 are a next row
 and are not part of this module.
"""
from __future__ import annotations

import numpy as np
from sklearn.metrics import (accuracy_score, classification_report, confusion_matrix,
                             f1_score)


def full_loss(predictions, y_test, verbose=True):
    """MOSI metrics (losses.py:276-315)."""
    predictions = np.asarray(predictions).flatten()
    y_test = np.asarray(y_test).flatten()
    mae = np.mean(np.absolute(predictions - y_test))
    corr = np.corrcoef(predictions, y_test)[0][1]
    mult = round(sum(np.round(predictions) == np.round(y_test)) / float(len(y_test)), 5)
    f_score = round(f1_score(np.round(predictions), np.round(y_test), average="weighted"), 5)
    true_label = (y_test >= 0)
    predicted_label = (predictions >= 0)
    accuracy = accuracy_score(true_label, predicted_label)
    confusion_mat = confusion_matrix(true_label, predicted_label)
    class_report = classification_report(true_label, predicted_label, digits=5, output_dict=True)
    if verbose:
        print("mae: {}".format(mae))
        print("corr: {}".format(corr))
        print("mult_acc: {}".format(mult))
        print("mult f_score: {}".format(f_score))
        print("Confusion Matrix :")
        print(confusion_mat)
        print("Classification Report :")
        print(classification_report(true_label, predicted_label, digits=5))
        print("Accuracy {}".format(accuracy))
    return {
        "mae": float(mae),
        "accuracy": float(accuracy),
        "corr": float(corr),
        "mult_acc": float(mult),
        "f_score": float(f_score),
        "confusion_matrix": confusion_mat.tolist(),
        "class_report": class_report,
    }


def iemocap_loss(predictions, y_test, verbose=True):
    """IEMOCAP metrics (losses.py:317-340)."""
    all_true_label = np.argmax(y_test, axis=1)
    all_predicted_label = np.argmax(predictions, axis=1)
    f_score = f1_score(all_true_label, all_predicted_label, average="weighted")
    accuracy = accuracy_score(all_true_label, all_predicted_label)
    confusion_mat = confusion_matrix(all_true_label, all_predicted_label)
    class_report = classification_report(all_true_label, all_predicted_label, digits=5,
                                         output_dict=True)
    if verbose:
        print("F1 score:", f_score)
        print("Accuracy:", accuracy)
        print("Confusion Matrix :")
        print(confusion_mat)
        print("Classification Report :")
        print(classification_report(all_true_label, all_predicted_label, digits=5))
    return {
        "accuracy": float(accuracy),
        "f_score": float(f_score),
        "confusion_matrix": confusion_mat.tolist(),
        "class_report": class_report,
    }


def pom_loss(predictions, y_test, verbose=True):
    """POM metrics, one value per label column (losses.py:342-366)."""
    predictions = np.asarray(predictions)
    y_test = np.asarray(y_test)
    mae = np.mean(np.absolute(predictions - y_test), axis=0)
    mae = [round(a, 3) for a in mae]
    corr = [round(np.corrcoef(predictions[:, i], y_test[:, i])[0][1], 3)
            for i in range(y_test.shape[1])]
    mult = [round(sum(np.round(predictions[:, i]) == np.round(y_test[:, i])) / float(len(y_test)), 3)
            for i in range(y_test.shape[1])]
    f_score = [round(f1_score(np.round(predictions[:, i]), np.round(y_test[:, i]),
                              average="weighted"), 5) for i in range(y_test.shape[1])]
    if verbose:
        print("mae:", mae)
        print("corr:", corr)
        print("mult_acc:", mult)
        print("f_score:", f_score)
    return {
        "mae": [float(x) for x in mae],
        "corr": [float(x) for x in corr],
        "mult_acc": [float(x) for x in mult],
        "f_score": [float(x) for x in f_score],
    }
